#include "g2o_utils.hpp"

#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
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

int parse_g2o(const std::string& fname, State& state, BearingObservationVector& bearings,
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
