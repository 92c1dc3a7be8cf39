#include "error.hpp"

#include "../../../include/bos.h"

namespace {
thread_local std::string g_last_error;
}

namespace bos {
int set_error(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}
}  // namespace bos

extern "C" const char* bos_last_error(void) { return g_last_error.c_str(); }
