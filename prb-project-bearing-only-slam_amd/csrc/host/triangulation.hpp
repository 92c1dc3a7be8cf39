// Landmark initial guess — mirror of slam/triangulation.hpp:8.
#pragma once

#include "observation.hpp"
#include "state.hpp"

namespace proj02 {

// slam/triangulation.cpp:5-19 (std::map => ascending landmark id)
BearingObservationsByLandmarkId subdivide_bearings_by_landmark_id(const BearingObservationVector& all);

// slam/triangulation.cpp:21-62: least squares over the rays [sin(th+a), -cos(th+a)] x = sin*px - cos*py,
// with the column-pivoted basic solution for a rank-1 system (one observation). verbose prints the
// reference's single-observation warning (:38-42).
LMPos triangulate_one_landmark(const State& state, const BearingObservationVector& observations, bool verbose);

// slam/triangulation.cpp:65-74: adds the triangulated landmarks to the state in ascending-id order.
void triangulate_landmarks(State& state, const BearingObservationVector& observations, bool verbose = true);

}  // namespace proj02
