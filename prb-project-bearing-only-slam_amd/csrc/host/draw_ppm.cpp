#include "draw_ppm.hpp"

#include <cmath>
#include <cstdio>

namespace proj02 {

namespace {

const unsigned char kPose[3] = {255, 0, 0};      // POSE_COLOR (BGR 0,0,255 in the reference)
const unsigned char kLm[3] = {0, 0, 255};        // LM_COLOR
const unsigned char kOdo[3] = {250, 0, 255};     // ODOMETRY_COLOR
constexpr int kPoseRadius = 4, kLmRadius = 2;

void to_px(const PpmImage& img, double x, double y, float bound, double& px, double& py) {
    px = (x + bound) / (2.0 * bound) * (img.w - 1);
    py = (img.h - 1) - (y + bound) / (2.0 * bound) * (img.h - 1);   // y up
}

void segment(PpmImage& img, double x0, double y0, double x1, double y1, const unsigned char c[3]) {
    const int n = (int)std::ceil(std::max(std::fabs(x1 - x0), std::fabs(y1 - y0))) + 1;
    if (n > 4 * (img.w + img.h)) return;   // off-image junk
    for (int i = 0; i <= n; ++i) {
        const double t = (double)i / n;
        img.set((int)std::lround(x0 + t * (x1 - x0)), (int)std::lround(y0 + t * (y1 - y0)), c);
    }
}

void circle(PpmImage& img, double cx, double cy, int r, const unsigned char c[3]) {
    const int n = 8 * r + 8;
    for (int i = 0; i < n; ++i) {
        const double a = 2.0 * M_PI * i / n;
        img.set((int)std::lround(cx + r * std::cos(a)), (int)std::lround(cy + r * std::sin(a)), c);
    }
}

}  // namespace

void draw_state_ppm(PpmImage& img, const State& state, const OdometryObservationVector& odometries, float bound) {
    if (!(bound > 0)) bound = 1;
    double px, py, qx, qy;
    for (const OdometryObservation& o : odometries) {
        const NEPose a = state.get_pose_by_id(o.get_source_id()), b = state.get_pose_by_id(o.get_dest_id());
        to_px(img, a.x, a.y, bound, px, py);
        to_px(img, b.x, b.y, bound, qx, qy);
        segment(img, px, py, qx, qy, kOdo);
    }
    for (const LMPos& l : state.landmarks_vec()) {
        to_px(img, l.x, l.y, bound, px, py);
        circle(img, px, py, kLmRadius, kLm);
    }
    for (const NEPose& p : state.poses_vec()) {
        to_px(img, p.x, p.y, bound, px, py);
        circle(img, px, py, kPoseRadius, kPose);
        segment(img, px, py, px + 2 * kPoseRadius * std::cos(p.theta), py - 2 * kPoseRadius * std::sin(p.theta), kPose);
    }
}

int write_ppm(const std::string& fname, const PpmImage& img) {
    FILE* f = std::fopen(fname.c_str(), "wb");
    if (!f) return -1;
    std::fprintf(f, "P6\n%d %d\n255\n", img.w, img.h);
    const size_t n = std::fwrite(img.rgb.data(), 1, img.rgb.size(), f);
    std::fclose(f);
    return n == img.rgb.size() ? 0 : -1;
}

}  // namespace proj02
