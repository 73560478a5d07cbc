// Kernel-argument block of the tfk MFMA implicit-GEMM engine (gemm.hip). Shared verbatim by the
// device code and the host bindings so the layout can never drift.
#pragma once
namespace tfk {
struct GemmParams {
  const void* A;
  const void* B;
  void* C;
  int M, N, K;
  long long lda, ldb, ldc;
  long long sA, sB, sC;  // batch strides (elements), batch = gridDim.y
  // conv geometry: X[Nimg][H][W][Cin] -> Y[Nimg][P][Q][Cout], filter R x S
  int Nimg, H, W, Cin, P, Q, Cout, R, S, sh, sw, ph, pw, dh, dw;
  float alpha, beta;
  const float* bias;   // [N] f32 or null
  const void* resid;   // [M][ldc] bf16 or null (added after activation)
  int act;             // 0 none, 1 relu, 2 gelu(tanh)
  float* stats;        // [shards][2][N] f32 (sum, sumsq) or null
  int stats_shards;
  int kt_per_split;
  long long split_stride;  // f32 elements between split-K slabs
  int tiles_n;
};
}  // namespace tfk
