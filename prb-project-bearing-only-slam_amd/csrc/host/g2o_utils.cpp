#include "g2o_utils.hpp"

#include <algorithm>
#include <array>
#include <cerrno>
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <thread>
#include <vector>

namespace proj02 {

namespace {

// Tokenizer over one line; numbers parsed with strtol/strtod (the reference uses stoi/stof and
// rounds values to float — values are kept in double here).
struct Line {
    const char* p;
    explicit Line(const char* s) : p(s) {}
    bool word(std::string& out) {
        while (*p == ' ' || *p == '\t' || *p == '\r' || *p == '\n') ++p;
        if (!*p) return false;
        const char* b = p;
        while (*p && *p != ' ' && *p != '\t' && *p != '\r' && *p != '\n') ++p;
        out.assign(b, p);
        return true;
    }
    bool integer(int& v) {
        std::string w;
        if (!word(w)) return false;
        char* end = nullptr;
        errno = 0;
        const long x = std::strtol(w.c_str(), &end, 10);
        if (end == w.c_str() || errno) return false;
        v = (int)x;
        return true;
    }
    bool real(double& v) {
        std::string w;
        if (!word(w)) return false;
        char* end = nullptr;
        v = std::strtod(w.c_str(), &end);
        return end != w.c_str();
    }
};

}  // namespace

int parse_g2o_simple(const std::string& fname, State& state, BearingObservationVector& bearings,
                     OdometryObservationVector& odometries, int& fixed_pose_id, float& bound) {
    bound = 0;
    fixed_pose_id = -1;
    FILE* f = std::fopen(fname.c_str(), "r");
    if (!f) return -1;
    std::vector<char> buf(1 << 16);
    std::string type;
    double fb = 0;   // bound accumulated in double, reported as float like the reference
    int rc = 0;
    while (std::fgets(buf.data(), (int)buf.size(), f)) {
        Line ln(buf.data());
        if (!ln.word(type)) continue;                                   // empty line (:113-116)
        if (type == "VERTEX_SE2") {                                     // :19-37
            int id; double x, y, th;
            if (!(ln.integer(id) && ln.real(x) && ln.real(y) && ln.real(th))) { rc = -2; break; }
            fb = std::max(fb, std::max(std::fabs(x), std::fabs(y)));
            state.add_pose(x, y, th, id);
        } else if (type == "VERTEX_XY") {                               // :40-56
            int id; double x, y;
            if (!(ln.integer(id) && ln.real(x) && ln.real(y))) { rc = -2; break; }
            fb = std::max(fb, std::max(std::fabs(x), std::fabs(y)));
            state.add_landmark(x, y, id);
        } else if (type == "FIX") {                                     // :59-65 (last one wins)
            int id;
            if (!ln.integer(id)) { rc = -2; break; }
            fixed_pose_id = id;
        } else if (type == "EDGE_SE2") {                                // :68-98
            int s, d; double x, y, th, u[6];
            if (!(ln.integer(s) && ln.integer(d) && ln.real(x) && ln.real(y) && ln.real(th))) { rc = -2; break; }
            bool ok = true;
            for (int k = 0; k < 6; ++k) ok = ok && ln.real(u[k]);
            if (!ok) { rc = -2; break; }
            Mat3 om;
            om(0, 0) = u[0]; om(0, 1) = u[1]; om(0, 2) = u[2];
            om(1, 0) = u[1]; om(1, 1) = u[3]; om(1, 2) = u[4];
            om(2, 0) = u[2]; om(2, 1) = u[4]; om(2, 2) = u[5];
            odometries.emplace_back(s, d, x, y, th, om);
        } else if (type == "EDGE_BEARING_SE2_XY") {                     // :101-110, omega = 1
            int p, l; double z;
            if (!(ln.integer(p) && ln.integer(l) && ln.real(z))) { rc = -2; break; }
            bearings.emplace_back(p, l, z);
        } else {
            std::cout << "Unrecognized " << type << std::endl;          // :118-120
        }
    }
    std::fclose(f);
    if (rc) return rc;
    bound = (float)fb + 3.0f;                                           // :124
    if (state.number_of_poses() == 0) std::cout << "Warning: no poses found. Stuff is likely to break." << std::endl;
    if (bearings.empty()) std::cout << "Warning: no bearing observations found. Stuff is likely to break." << std::endl;
    return 0;
}

namespace {

// ---- parallel parser: the file is read at once, cut into chunks at line starts, each chunk parsed
// by its own thread into per-chunk vectors (std::from_chars: correctly rounded like strtod), and
// the chunks merged in file order, so the result equals the line-by-line parser's.
struct Tok {
    const char* p;
    const char* e;
    bool next(const char*& b, const char*& t) {
        while (p < e && (*p == ' ' || *p == '\t' || *p == '\r')) ++p;
        if (p >= e) return false;
        b = p;
        while (p < e && *p != ' ' && *p != '\t' && *p != '\r') ++p;
        t = p;
        return true;
    }
    // a token parsed like strtol / strtod on it (leading '+' allowed, trailing junk ignored)
    bool integer(int& v) {
        const char *b, *t;
        if (!next(b, t)) return false;
        if (*b == '+') ++b;
        long x = 0;
        const auto r = std::from_chars(b, t, x);
        if (r.ec != std::errc() || x < INT32_MIN || x > INT32_MAX) return false;
        v = (int)x;
        return true;
    }
    bool real(double& v) {
        const char *b, *t;
        if (!next(b, t)) return false;
        if (*b == '+') ++b;
        const auto r = std::from_chars(b, t, v);
        if (r.ec == std::errc::result_out_of_range) v = std::strtod(std::string(b, t).c_str(), nullptr);   // +-inf / 0
        return r.ec == std::errc() || r.ec == std::errc::result_out_of_range;
    }
};

struct ChunkOut {
    std::vector<std::pair<int, std::array<double, 3>>> poses;
    std::vector<std::pair<int, std::array<double, 2>>> landmarks;
    OdometryObservationVector odometries;
    BearingObservationVector bearings;
    std::vector<std::string> unknown;
    int fix = -1;
    double fb = 0;
    bool bad = false;
};

bool tok_is(const char* b, const char* t, const char* w) {
    const size_t n = std::strlen(w);
    return (size_t)(t - b) == n && std::memcmp(b, w, n) == 0;
}

void parse_chunk(const char* p, const char* e, ChunkOut& o) {
    while (p < e && !o.bad) {
        const char* le = (const char*)std::memchr(p, '\n', (size_t)(e - p));
        if (!le) le = e;
        Tok ln{p, le};
        p = le + 1;
        const char *b, *t;
        if (!ln.next(b, t)) continue;                                   // empty line (:113-116)
        if (tok_is(b, t, "VERTEX_SE2")) {                               // :19-37
            int id; double x, y, th;
            if (!(ln.integer(id) && ln.real(x) && ln.real(y) && ln.real(th))) { o.bad = true; break; }
            o.fb = std::max(o.fb, std::max(std::fabs(x), std::fabs(y)));
            o.poses.push_back({id, {x, y, th}});
        } else if (tok_is(b, t, "VERTEX_XY")) {                         // :40-56
            int id; double x, y;
            if (!(ln.integer(id) && ln.real(x) && ln.real(y))) { o.bad = true; break; }
            o.fb = std::max(o.fb, std::max(std::fabs(x), std::fabs(y)));
            o.landmarks.push_back({id, {x, y}});
        } else if (tok_is(b, t, "FIX")) {                               // :59-65 (last one wins)
            int id;
            if (!ln.integer(id)) { o.bad = true; break; }
            o.fix = id;
        } else if (tok_is(b, t, "EDGE_SE2")) {                          // :68-98
            int s, d; double x, y, th, u[6];
            if (!(ln.integer(s) && ln.integer(d) && ln.real(x) && ln.real(y) && ln.real(th))) { o.bad = true; break; }
            bool ok = true;
            for (int k = 0; k < 6; ++k) ok = ok && ln.real(u[k]);
            if (!ok) { o.bad = true; break; }
            Mat3 om;
            om(0, 0) = u[0]; om(0, 1) = u[1]; om(0, 2) = u[2];
            om(1, 0) = u[1]; om(1, 1) = u[3]; om(1, 2) = u[4];
            om(2, 0) = u[2]; om(2, 1) = u[4]; om(2, 2) = u[5];
            o.odometries.emplace_back(s, d, x, y, th, om);
        } else if (tok_is(b, t, "EDGE_BEARING_SE2_XY")) {               // :101-110, omega = 1
            int ps, l; double z;
            if (!(ln.integer(ps) && ln.integer(l) && ln.real(z))) { o.bad = true; break; }
            o.bearings.emplace_back(ps, l, z);
        } else {
            o.unknown.emplace_back(b, t);                               // :118-120
        }
    }
}

}  // namespace

int g_g2o_line_parser = 0;

int parse_g2o(const std::string& fname, State& state, BearingObservationVector& bearings,
              OdometryObservationVector& odometries, int& fixed_pose_id, float& bound) {
    if (g_g2o_line_parser) return parse_g2o_simple(fname, state, bearings, odometries, fixed_pose_id, bound);
    bound = 0;
    fixed_pose_id = -1;
    FILE* f = std::fopen(fname.c_str(), "rb");
    if (!f) return -1;
    std::vector<char> buf;
    {
        std::fseek(f, 0, SEEK_END);
        const long n = std::ftell(f);
        std::fseek(f, 0, SEEK_SET);
        if (n < 0) { std::fclose(f); return -1; }
        buf.resize((size_t)n);
        if (n > 0 && std::fread(buf.data(), 1, (size_t)n, f) != (size_t)n) { std::fclose(f); return -1; }
    }
    std::fclose(f);
    const char* base = buf.data();
    const size_t n = buf.size();
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const int nt = (int)std::min<size_t>(std::min(16u, hw), std::max<size_t>(1, n >> 20));   // >= 1 MiB per chunk
    std::vector<size_t> cut(nt + 1, n);
    cut[0] = 0;
    for (int c = 1; c < nt; ++c) {
        size_t q = std::max(cut[c - 1], n * c / nt);
        while (q < n && q > 0 && base[q - 1] != '\n') ++q;   // chunks start at line starts
        cut[c] = q;
    }
    std::vector<ChunkOut> out(nt);
    std::vector<std::thread> th;
    for (int c = 1; c < nt; ++c) th.emplace_back(parse_chunk, base + cut[c], base + cut[c + 1], std::ref(out[c]));
    parse_chunk(base + cut[0], base + cut[1], out[0]);
    for (std::thread& t : th) t.join();
    double fb = 0;
    for (const ChunkOut& o : out) {
        if (o.bad) return -2;
        for (const auto& q : o.poses) state.add_pose(q.second[0], q.second[1], q.second[2], q.first);
        for (const auto& q : o.landmarks) state.add_landmark(q.second[0], q.second[1], q.first);
        odometries.insert(odometries.end(), o.odometries.begin(), o.odometries.end());
        bearings.insert(bearings.end(), o.bearings.begin(), o.bearings.end());
        for (const std::string& u : o.unknown) std::cout << "Unrecognized " << u << std::endl;
        if (o.fix >= 0) fixed_pose_id = o.fix;
        fb = std::max(fb, o.fb);
    }
    bound = (float)fb + 3.0f;                                           // :124
    if (state.number_of_poses() == 0) std::cout << "Warning: no poses found. Stuff is likely to break." << std::endl;
    if (bearings.empty()) std::cout << "Warning: no bearing observations found. Stuff is likely to break." << std::endl;
    return 0;
}

int parse_g2o(const std::string& fname, State& state, BearingObservationVector& bearings, int& fixed_pose_id,
              float& bound) {
    OdometryObservationVector unused;
    return parse_g2o(fname, state, bearings, unused, fixed_pose_id, bound);
}

int write_g2o(const std::string& fname, const State& state, const BearingObservationVector& bearings,
              const OdometryObservationVector& odometries, int fixed_pose_id, bool with_landmarks) {
    FILE* f = std::fopen(fname.c_str(), "w");
    if (!f) return -1;
    const NEPoseVector& P = state.poses_vec();
    const AssociationVec& pid = state.pose_ids();
    for (size_t i = 0; i < P.size(); ++i) {
        const EPose e = t2v(P[i]);
        std::fprintf(f, "VERTEX_SE2 %d %.17g %.17g %.17g\n", pid[i], e.x, e.y, e.z);
    }
    if (with_landmarks) {
        const LMPosVector& L = state.landmarks_vec();
        const AssociationVec& lid = state.landmark_ids();
        for (size_t j = 0; j < L.size(); ++j) std::fprintf(f, "VERTEX_XY %d %.17g %.17g\n", lid[j], L[j].x, L[j].y);
    }
    if (fixed_pose_id >= 0) std::fprintf(f, "FIX %d\n", fixed_pose_id);
    for (const OdometryObservation& o : odometries) {
        const EPose z = o.get_transformation();
        const Mat3 m = o.get_omega();
        std::fprintf(f, "EDGE_SE2 %d %d %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g\n", o.get_source_id(),
                     o.get_dest_id(), z.x, z.y, z.z, m(0, 0), m(0, 1), m(0, 2), m(1, 1), m(1, 2), m(2, 2));
    }
    for (const BearingObservation& b : bearings)
        std::fprintf(f, "EDGE_BEARING_SE2_XY %d %d %.17g %.17g\n", b.get_pose_id(), b.get_lm_id(), b.get_bearing(),
                     b.get_omega() * 57295.779513082323);
    std::fclose(f);
    return 0;
}

}  // namespace proj02
