// Arguments of the finalize-in-apply BatchNorm kernels (bn.hip), shared with the host bindings.
#pragma once

namespace tfk {

// Forward finalize of one BN (stats [shards][2][C]); stats == nullptr: apply with the given scale/shift.
struct BnFin {
  const float* stats;
  const float* gamma;
  const float* beta;
  float* run_mean;
  float* run_var;
  float* mean;
  float* invstd;
  float* scale;  // in (stats == nullptr) or out
  float* shift;
  float eps, momentum;
  int shards;
};

// Backward finalize of one BN from sums [shards][3][C] (sum dz, sum dz*xhat, sum dz*xhat2).
struct BnBwdFin {
  const float* gamma;
  const float* mean;
  const float* invstd;
  float* dgamma;
  float* dbeta;
};

}  // namespace tfk
