// tfk "w128" GEMM engine for gfx950: 256x256 block tile, 4 waves (ONE per SIMD), each wave owning
// a 128x128 output tile = 8x8 fragments of v_mfma_f32_16x16x32_bf16 -> 256 accumulator registers in
// the AGPR half of the unified 512-entry file (the hipBLASLt MT256x256x64 layout;
// profiles/pmc_pingpong_vs_hipblaslt_8192_r2.txt: same MFMA busy cycles as our 16-wave 256x256
// kernel at a third of the wave cycles and 1/20 of the wait time).
//
// Why: per 64-deep K-tile a 64x64 wave tile reads 16 KiB of fragments for 32 MFMAs; a 128x128 one
// reads 32 KiB for 128 MFMAs -- half the LDS traffic per FLOP, and 4 instead of 16 waves at the
// block barrier. With one wave per SIMD nothing else hides a stall, so the schedule is explicit:
//
//   K-tile t (stage s = t & 1, two 64-KiB LDS stages, operand images of gemm_g4.hip / g4_loader.h):
//     issue the LDS-DMA of tile t+1 into stage s^1
//     read B k-half-1 fragments (8 x 16 B)                      -- land during k-half 0
//     k-half 0: for each of 8 A fragments: read A[i+1], 8 MFMAs  -- one A read ahead (128 cycles)
//     k-half 1: the same, but BEFORE the last A fragment's MFMAs:
//        s_waitcnt vmcnt(0) lgkmcnt(0); s_barrier      (tile t+1 landed, stage s fully read)
//        read tile t+1's B k-half-0 fragments and A[0]  -- land under those last 8 MFMAs
//   so the LDS latency after the barrier hides under 128 MFMA cycles instead of stalling the SIMD,
//   and each K-tile costs one barrier among 4 waves.
// sched_barrier(0) fences keep the compiler from moving MFMAs across the barrier point.
//
// Included by gemm_w128*.hip with W128_NS (namespace), W128_V2 (1: single-basic-block loop body),
// W128_SGB (sched_group_barrier pipeline) and per-file hipcc flags (scheduler strategy): the
// variants are A/B'd on the GPU through tfk_w128_set(variant).
#pragma once
#include "common.h"
#include "gemm_params.h"
#include "gemm_epilogue.h"
#include "g4_loader.h"

namespace tfk {
namespace W128_NS {

using g4::BK;
using g4::Loader;
using g4::frag;
using g4::KIN;
using g4::KOUT;
using g4::CONV_WGRAD;

constexpr int BM = 256, BN = 256, NW = 4, NTH = 256, WGM = 2, WGN = 2, FM = 8, FN = 8;
constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE = A_BYTES + B_BYTES;
constexpr bool SGB = W128_SGB;

template <int AM, int BMD, int EPI>
__global__ __launch_bounds__(NTH, 1) void w128_kernel(GemmParams p) {
  constexpr int LBM = BMD == 2 ? CONV_WGRAD : BMD;
  constexpr bool AKO = (AM == KOUT), BKO = (LBM == KOUT || LBM == CONV_WGRAD);
  constexpr int MAIN = 2 * STAGE, EPIB = epi_lds_bytes<BM, BN, WGM>();
  __shared__ __attribute__((aligned(16))) char smem[MAIN > EPIB ? MAIN : EPIB];

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w / WGN, wn = w % WGN;
  const int bz = blockIdx.y;

  const int tiles_m = (p.M + BM - 1) / BM;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  constexpr int GM = 4;
  const int grp = tile / (GM * p.tiles_n), first_m = grp * GM;
  const int gm = min(GM, tiles_m - first_m), inr = tile - grp * GM * p.tiles_n;
  const int m0 = (first_m + inr % gm) * BM, n0 = (inr / gm) * BN;

  const int nkt = (p.K + BK - 1) / BK;
  const int kt0 = blockIdx.z * p.kt_per_split;
  const int kt1 = min(nkt, kt0 + p.kt_per_split);

  const char* Ab = (const char*)p.A + (long long)bz * p.sA * 2 + (AKO ? (long long)m0 * 2 : (long long)m0 * p.lda * 2);
  const char* Bb = (const char*)p.B + (long long)bz * p.sB * 2 +
                   (LBM == CONV_WGRAD ? 0LL : BKO ? (long long)n0 * 2 : (long long)n0 * p.ldb * 2);
  const long long a_step = AKO ? (long long)BK * p.lda * 2 : BK * 2;
  const long long b_step = BKO ? (long long)BK * p.ldb * 2 : BK * 2;
  const int lim_a = p.M - m0, lim_b = p.N - n0;

  Loader<BM, AM, NW, false> la;
  Loader<BN, LBM, NW> lb;
  la.init(p, lane, w, p.lda, m0, p.M);
  lb.init(p, lane, w, p.ldb, n0, p.N);

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto stage_ptr = [&](int s) { return smem + s * STAGE; };
  const int ar = wm * 128, bc = wn * 128;

  bf16x8 b0[FN], b1[FN], a_cur;
  if (kt0 < kt1) {
    la.issue(p, Ab, a_step, kt0, lim_a, stage_ptr(0), w, lane);
    lb.issue(p, Bb, b_step, kt0, lim_b, stage_ptr(0) + A_BYTES, w, lane);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
#pragma unroll
  for (int j = 0; j < FN; ++j) b0[j] = frag<BKO>(stage_ptr(0) + A_BYTES, bc + j * 16, 0);
  a_cur = frag<AKO>(stage_ptr(0), ar, 0);

#if W128_V2
  // The loop body is ONE basic block (no `if (more)`: on the last K-tile the DMA gets lim 0 -- every
  // lane out of range, zero-filled, no memory traffic -- and the barrier + next-tile reads run on
  // data nobody uses), so the sched_group_barrier pipeline below can place every instruction:
  //   k-half 0, per A fragment i: 2 LDS-DMA issues, read B k1 fragment i, read A[i+1]; 8 MFMAs
  //   k-half 1, per A fragment i < 7: read A[i+1]; 8 MFMAs
  // (the compiler's own schedule issued each read right before its consumer and exposed the LDS
  // latency twice per 16 MFMAs).
#pragma unroll 1
  for (int kt = kt0; kt < kt1; ++kt) {
    const int s = (kt - kt0) & 1;
    const char* As = stage_ptr(s);
    const char* Bs = As + A_BYTES;
    const bool more = kt + 1 < kt1;  // block-uniform
    {
      char* nx = stage_ptr(s ^ 1);
      la.issue(p, Ab, a_step, kt + 1, more ? lim_a : 0, nx, w, lane);
      lb.issue(p, Bb, b_step, kt + 1, more ? lim_b : 0, nx + A_BYTES, w, lane);
    }
    // k-half 0
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      b1[i] = frag<BKO>(Bs, bc + i * 16, 1);
      const bf16x8 a_nx = frag<AKO>(As, ar + ((i + 1) & (FM - 1)) * 16, i + 1 < FM ? 0 : 1);
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b0[j], a_cur, acc[i][j], 0, 0, 0);
      a_cur = a_nx;
    }
    // k-half 1
#pragma unroll
    for (int i = 0; i < FM - 1; ++i) {
      const bf16x8 a_nx = frag<AKO>(As, ar + (i + 1) * 16, 1);
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b1[j], a_cur, acc[i][j], 0, 0, 0);
      a_cur = a_nx;
    }
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      if (SGB) __builtin_amdgcn_sched_group_barrier(0x020, 2, 0);  // VMEM (LDS-DMA)
      if (SGB) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // DS read
      if (SGB) __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);  // MFMA
    }
#pragma unroll
    for (int i = 0; i < FM - 1; ++i) {
      if (SGB) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      if (SGB) __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    {
      const char* An = stage_ptr(s ^ 1);
#pragma unroll
      for (int j = 0; j < FN; ++j) b0[j] = frag<BKO>(An + A_BYTES, bc + j * 16, 0);
      const bf16x8 a_nx = frag<AKO>(An, ar, 0);
#pragma unroll
      for (int j = 0; j < FN; ++j)
        acc[FM - 1][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b1[j], a_cur, acc[FM - 1][j], 0, 0, 0);
      a_cur = a_nx;
    }
    __builtin_amdgcn_sched_barrier(0);
  }
#else
#pragma unroll 1
  for (int kt = kt0; kt < kt1; ++kt) {
    const int s = (kt - kt0) & 1;
    const char* As = stage_ptr(s);
    const char* Bs = As + A_BYTES;
    const bool more = kt + 1 < kt1;  // block-uniform
    if (more) {
      char* nx = stage_ptr(s ^ 1);
      la.issue(p, Ab, a_step, kt + 1, lim_a, nx, w, lane);
      lb.issue(p, Bb, b_step, kt + 1, lim_b, nx + A_BYTES, w, lane);
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) b1[j] = frag<BKO>(Bs, bc + j * 16, 1);
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const bf16x8 a_nx = frag<AKO>(As, ar + ((i + 1) & (FM - 1)) * 16, i + 1 < FM ? 0 : 1);
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b0[j], a_cur, acc[i][j], 0, 0, 0);
      a_cur = a_nx;
    }
#pragma unroll
    for (int i = 0; i < FM - 1; ++i) {
      const bf16x8 a_nx = frag<AKO>(As, ar + (i + 1) * 16, 1);
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b1[j], a_cur, acc[i][j], 0, 0, 0);
      a_cur = a_nx;
    }
    bf16x8 a_nx = a_cur;
    if (more) {
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      const char* An = stage_ptr(s ^ 1);
#pragma unroll
      for (int j = 0; j < FN; ++j) b0[j] = frag<BKO>(An + A_BYTES, bc + j * 16, 0);
      a_nx = frag<AKO>(An, ar, 0);
    }
#pragma unroll
    for (int j = 0; j < FN; ++j)
      acc[FM - 1][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b1[j], a_cur, acc[FM - 1][j], 0, 0, 0);
    a_cur = a_nx;
  }
#endif
  __syncthreads();
  gemm_epilogue<BM, BN, NTH, WGM, EPI, 4>(p, acc, smem, m0, n0, bz);
}

}  // namespace W128_NS
}  // namespace tfk

