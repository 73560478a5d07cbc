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
  // Fused BatchNorm-backward reduction over the final bf16 output dA (bf16 epilogue only, N%8==0):
  //   dz = dA * mask,  mask = bn_amask ? bit : bn_relu ? (y*scale+shift > 0) : 1
  //   (bn_amask: packed relu mask of the activation, bit e of byte i/8 = a[i+e] > 0, as the
  //   forward's bn_apply writes it -- 1 byte per 8-element chunk instead of 16)
  //   bn_sums[shard][0][n] += dz,  [1][n] += dz*(y-mean)*invstd,  [2][n] += dz*(y2-mean2)*invstd2
  const void* bn_y;
  const unsigned char* bn_amask;
  const float* bn_mean;
  const float* bn_invstd;
  const float* bn_scale;
  const float* bn_shift;
  int bn_relu;
  // store dz (= dA * mask, the value the sums see) instead of dA: the consumer of dA is the BN
  // backward, which then needs neither the mask nor a separate residual-gradient output (for an
  // identity shortcut d(residual) = dz)
  int bn_store_dz;
  const void* bn_y2;
  const float* bn_mean2;
  const float* bn_invstd2;
  float* bn_sums;
  int bn_shards;
  // bf16 epilogue extras: aux = pre-activation copy of C (e.g. GELU input saved for backward);
  // dact_src/dact: C = (A*B) * act'(dact_src) (activation backward fused into a dgrad GEMM).
  void* aux;
  const void* dact_src;
  int dact;
  // relu bitmasks instead of bf16 pre-activations: aux_bits -> aux is uint8 [rows][ldc/8], bit e of
  // byte (m*ldc + n)/8 = (pre-activation of column n+e > 0); dact_bits -> dact_src is such a mask
  // and the activation backward is relu' (1/16 of the bytes of a bf16 z, written and read)
  int aux_bits;
  int dact_bits;
  // EXT epilogue: += column sums of the bf16 output before any residual add ([N] f32; the bias
  // gradient of the layer that consumes C, e.g. FFN1's from FFN2's dgrad -- no separate column pass)
  float* colsum;
  // inverted dropout after the activation, before the residual add; mask = hash(seed, m*N + n),
  // identical to misc.hip's dropout kernel on the contiguous [M][N] output (backward regenerates it)
  float drop_p, drop_scale;
  unsigned long long drop_seed;            // per-site salt
  const unsigned long long* drop_seed_key; // per-step device key (common.h eff_seed) or null
  // MX-fp8 engine (fp8.hip): e8m0 block scales, [rows][K/32] bytes, one per 32 K-elements
  const void* a_scale;
  const void* b_scale;
  // bf16-epilogue row maps (strided-conv dgrad, gemm_epilogue.h out_row/resid_row):
  //  out-map (om_hp > 0): GEMM row m = (n, h', w') of an [om_hp][om_wp] phase grid is output row
  //    (n, h'*om_sh + om_a, w'*om_sw + om_b) of the [om_h][om_w] grid (C, resid, bn_* share it);
  //  resid sub-sampling (rs_sh > 0): output row (n, h, w) of [rs_h][rs_w] reads resid row
  //    (n, h/rs_sh, w/rs_sw) of [rs_p][rs_q] on the stride lattice and no resid elsewhere.
  int om_hp, om_wp, om_h, om_w, om_sh, om_sw, om_a, om_b;
  int rs_h, rs_w, rs_p, rs_q, rs_sh, rs_sw;
  // LDS-DMA conv weight-gradient gather (gemm_g4.hip): magic-number division of a pixel index by
  // Q and P*Q ((umulhi(x, mul) + x) >> shift, x < 2^31), filled by the g4 host launcher
  unsigned fd_q_mul, fd_pq_mul;
  int fd_q_shift, fd_pq_shift;
  // EPI_BF16_EXT_MX (MX-fp8 engine): MX copies of the final bf16 output C [M][N] for the next GEMMs
  // -- row blocks (mx_qr [M][N] e4m3, mx_sr [M][N/32] e8m0) and column blocks (mx_qc [N][M],
  // mx_sc [N][M/32]) -- quantized from the LDS C tile (M, N % 32 == 0, ldc == N). mx_skip_c: no
  // bf16 C store (its only consumers read the MX copies).
  void* mx_qr;
  void* mx_sr;
  void* mx_qc;
  void* mx_sc;
  int mx_skip_c;
};
}  // namespace tfk
