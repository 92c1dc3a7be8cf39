// g2o I/O — mirror of utils/g2o_utils.hpp:29 (parse_g2o) plus a writer the reference lacks
// (SURVEY.md §5 checkpoint/resume: the final state as a g2o file).
//
// Accepted lines (utils/g2o_utils.hpp:11-22):
//   VERTEX_SE2 id x y theta
//   VERTEX_XY id x y
//   FIX id
//   EDGE_SE2 i j x y theta <6 upper-triangular omega values, row-major>
//   EDGE_BEARING_SE2_XY id_pose id_landmark bearing <ignored information column>
#pragma once

#include <string>

#include "observation.hpp"
#include "state.hpp"

namespace proj02 {

// utils/g2o_utils.cpp:10-146. Returns 0 on success, -1 if the file cannot be opened, -2 on a
// malformed number (the reference would throw std::invalid_argument from stoi/stof).
// Unknown tokens print "Unrecognized <tok>" and are skipped (:129-131); bound gets +3 (:135).
int parse_g2o(const std::string& fname, State& state, BearingObservationVector& bearings,
              OdometryObservationVector& odometries, int& fixed_pose_id, float& bound);

// The line-by-line form of parse_g2o (parse_g2o reads the file at once and parses chunks in
// parallel, merged in file order; BOS_G2O_SIMPLE=1 selects this one instead).
// Test hook (bos_debug_set_g2o_parser): nonzero makes parse_g2o use the line-by-line form.
extern int g_g2o_line_parser;
int parse_g2o_simple(const std::string& fname, State& state, BearingObservationVector& bearings,
                     OdometryObservationVector& odometries, int& fixed_pose_id, float& bound);

// utils/g2o_utils.cpp:5-8 (legacy overload without odometry)
int parse_g2o(const std::string& fname, State& state, BearingObservationVector& bearings, int& fixed_pose_id,
              float& bound);

// Writes VERTEX_SE2 (+ VERTEX_XY if with_landmarks), FIX, EDGE_SE2 and EDGE_BEARING_SE2_XY lines.
int write_g2o(const std::string& fname, const State& state, const BearingObservationVector& bearings,
              const OdometryObservationVector& odometries, int fixed_pose_id, bool with_landmarks);

}  // namespace proj02
