// Headless rendering of a SLAM state to a binary PPM image: the OpenCV window of the reference
// (utils/draw_utils.cpp: poses as red circles with a heading ray, landmarks as blue circles,
// odometry as purple segments, the world [-bound, bound]^2 mapped to the image with y up),
// without OpenCV.
#pragma once

#include <string>

#include "observation.hpp"
#include "state.hpp"

namespace proj02 {

struct PpmImage {
    int w = 0, h = 0;
    std::vector<unsigned char> rgb;
    PpmImage(int width, int height) : w(width), h(height), rgb(3 * (size_t)width * height, 255) {}
    void set(int x, int y, const unsigned char c[3]) {
        if (x < 0 || x >= w || y < 0 || y >= h) return;
        unsigned char* p = &rgb[3 * ((size_t)y * w + x)];
        p[0] = c[0]; p[1] = c[1]; p[2] = c[2];
    }
};

// draw_state (utils/draw_utils.cpp): odometry, landmarks, poses
void draw_state_ppm(PpmImage& img, const State& state, const OdometryObservationVector& odometries, float bound);
int write_ppm(const std::string& fname, const PpmImage& img);

}  // namespace proj02
