// Thread-local last-error string shared by both halves of the C ABI (bos_last_error()).
#pragma once

#include <string>

namespace bos {
int set_error(int code, const std::string& msg);
}
