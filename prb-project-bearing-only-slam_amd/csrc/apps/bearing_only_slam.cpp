// Headless drop-in for executables/bearing_only_slam.cpp (reference :40-116).
// Usage: bearing_only_slam <dataset_fname> [--iters N] [--fp32] [--dense|--schur] [--dump out.g2o]
//                          [--ppm out.ppm] [--quiet]
// Same flow as the reference's main: parse_g2o, default the fixed pose, triangulate the
// landmarks, construct the Solver, then iterate (the reference's Tab press = 50 iterations,
// :93-99). The OpenCV window is replaced by a per-iteration chi^2 line, an optional g2o dump and
// an optional PPM rendering of the initial and final states (utils/draw_utils.cpp without OpenCV).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>

#include "../host/draw_ppm.hpp"
#include "../host/g2o_utils.hpp"
#include "../host/solver.hpp"
#include "../host/triangulation.hpp"

using namespace proj02;

int main(int argc, char** argv) {
    if (argc < 2) {
        std::cout << "usage: bearing_only_slam <dataset_fname> [--iters N] [--fp32] [--dense|--schur] [--dump out.g2o] "
                     "[--ppm out.ppm] [--quiet]"
                  << std::endl;
        return 1;
    }
    int iters = 50;
    bool quiet = false;
    std::string dump, ppm;
    bos_options opt;
    bos_default_options(&opt);
    for (int i = 2; i < argc; ++i) {
        if (!std::strcmp(argv[i], "--iters") && i + 1 < argc) iters = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--fp32")) opt.precision = BOS_FP32;
        else if (!std::strcmp(argv[i], "--dense")) opt.solver = BOS_SOLVER_DENSE_CHOL;
        else if (!std::strcmp(argv[i], "--schur")) opt.solver = BOS_SOLVER_SCHUR;
        else if (!std::strcmp(argv[i], "--dump") && i + 1 < argc) dump = argv[++i];
        else if (!std::strcmp(argv[i], "--ppm") && i + 1 < argc) ppm = argv[++i];
        else if (!std::strcmp(argv[i], "--quiet")) quiet = true;
        else { std::cerr << "unknown argument " << argv[i] << std::endl; return 1; }
    }
    State state(300, 200);
    BearingObservationVector bearings;
    OdometryObservationVector odometries;
    int fixed_pose_id = -1;
    float bound = 0;
    if (parse_g2o(argv[1], state, bearings, odometries, fixed_pose_id, bound)) {
        std::cerr << "cannot read " << argv[1] << std::endl;
        return 1;
    }
    if (fixed_pose_id < 0) fixed_pose_id = state.default_pose_id();
    triangulate_landmarks(state, bearings, !quiet);
    auto render = [&](const State& st, const std::string& path) {
        PpmImage img(800, 800);
        draw_state_ppm(img, st, odometries, bound);
        if (write_ppm(path, img)) std::cerr << "cannot write " << path << std::endl;
    };
    if (!ppm.empty()) render(state, ppm.substr(0, ppm.rfind('.')) + "_initial.ppm");
    try {
        Solver solver(state, bearings, odometries, fixed_pose_id, &opt);
        for (int it = 0; it < iters; ++it) {
            solver.step();
            const bos_step_stats& s = solver.last_stats();
            if (!quiet)
                std::printf("iter %3d  chi2 %.9g  robust %d  max|dx| %.3g  J+H %.3f ms  solve %.3f ms\n", it, s.chi2,
                            s.n_robust, s.max_abs_dx, s.t_linearize_ms, s.t_solve_ms);
        }
        if (!ppm.empty()) render(solver.state, ppm);
        if (!dump.empty() && write_g2o(dump, solver.state, bearings, odometries, fixed_pose_id, true)) {
            std::cerr << "cannot write " << dump << std::endl;
            return 1;
        }
    } catch (const std::exception& e) {
        std::cerr << e.what() << std::endl;
        return 2;
    }
    return 0;
}
