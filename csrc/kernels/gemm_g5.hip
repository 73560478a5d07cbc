// tfk "g5" GEMM engine for gfx950: 256x256 output tile, ONE barrier per K-tile, operand fragments
// of the next K-half read while the MFMAs of the current one run.
//
// Why (profiles/perf_log_r4.md): the g4 256x256 tile (16 waves) re-reads its k-half-0 fragments
// right after the end-of-tile barrier, so every K-tile opens with an LDS-latency bubble; the g8
// ping-pong schedule pays 8 barriers per K-tile. Here the barrier sits in the MIDDLE of a K-tile:
//
//   phase A (k-half 0 of tile t): MFMAs on R0 (read during the previous phase B)
//                                 || ds_reads of tile t's k-half 1 -> R1
//   s_waitcnt vmcnt(0) lgkmcnt(0)  (tile t+1's LDS-DMA landed; every read of stage t&1 retired)
//   barrier                        (all waves: tile t+1 visible, stage t&1 free)
//   phase B (k-half 1 of tile t): MFMAs on R1
//                                 || LDS-DMA of tile t+2 into stage t&1 (just freed)
//                                 || ds_reads of tile t+1's k-half 0 -> R0
//
// so the MFMA pipe always has a full K-half of independent work queued across the barrier, the
// DMA of a tile has a whole K-tile of MFMAs to land in, and a stage is overwritten only after the
// barrier that follows the last read of it ("restage a buffer only after an lgkmcnt + barrier").
// Inside each phase the ds_reads (and the DMA pieces) are spread between the MFMAs with
// __builtin_amdgcn_sched_group_barrier, so the wave never bursts its LDS traffic.
//
// Waves: WGM x WGN, each owning a (256/WGM) x (256/WGN) sub-tile of 16x16 fragments:
//   <2, 2>: 4 waves (one per SIMD), 128x128 each, 256 AGPR accumulators (hipBLASLt's
//           MT256x256x64 geometry);
//   <2, 4>: 8 waves (two per SIMD), 128x64 each.
// Operand images, LDS-DMA loaders and fragment readers are the g4 engine's (g4_loader.h); the
// epilogue is the shared LDS-staged one (gemm_epilogue.h).
#include "common.h"
#include "gemm_params.h"
#include "gemm_epilogue.h"
#include "g4_loader.h"

namespace tfk {
namespace g5 {

using g4::BK;
using g4::CONV_FWD;
using g4::frag;
using g4::KIN;
using g4::KOUT;
using g4::Loader;

constexpr int BM = 256, BN = 256;
constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE = A_BYTES + B_BYTES;  // 64 KiB

// Interleave NR reads (DS read group) and ND DMA pieces (VMEM group) between NM MFMAs.
template <int NM, int NR, int ND>
__device__ __forceinline__ void interleave() {
  constexpr int SLOTS = NR > ND ? NR : ND;
  constexpr int PER = NM / SLOTS, REM = NM - PER * SLOTS;
#pragma unroll
  for (int s = 0; s < SLOTS; ++s) {
    if (s < NR) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
    if (s < ND) __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);  // VMEM (LDS-DMA piece)
    __builtin_amdgcn_sched_group_barrier(0x008, PER, 0);            // MFMA
  }
  if (REM) __builtin_amdgcn_sched_group_barrier(0x008, REM, 0);
}

// SCHED 0: each phase's reads / DMA pieces are spread between its MFMAs by sched_group_barrier;
// SCHED 1: the phase is written as fixed slots {MFMAs, one DMA piece, one fragment read} fenced by
// sched_barrier, MFMAs first -- so right after the barrier the MFMA pipe restarts at once instead of
// behind the DMA address setup the scheduler otherwise hoists there.
template <int AM, int BMD, int EPI, int WGM, int WGN, int SCHED = 0>
__global__ __launch_bounds__(WGM * WGN * 64, 1) void g5_kernel(GemmParams p) {
  constexpr int NW = WGM * WGN, NT = NW * 64;
  constexpr int TM = BM / WGM, TN = BN / WGN, FM = TM / 16, FN = TN / 16;
  constexpr bool AKO = (AM == KOUT), BKO = (BMD == KOUT);
  constexpr int MAIN = 2 * STAGE, EPIB = epi_lds_bytes<BM, BN, WGM>();
  __shared__ __attribute__((aligned(16))) char smem[MAIN > EPIB ? MAIN : EPIB];

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w / WGN, wn = w % WGN;
  const int bz = blockIdx.y;

  // tile order: XCD remap, then GROUP_M = 4 inside each XCD's contiguous range (as g4)
  const int tiles_m = (p.M + BM - 1) / BM;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  constexpr int GM = 4;
  const int grp = tile / (GM * p.tiles_n), first_m = grp * GM;
  const int gm = min(GM, tiles_m - first_m), inr = tile - grp * GM * p.tiles_n;
  const int m0 = (first_m + inr % gm) * BM, n0 = (inr / gm) * BN;

  const int nkt = (p.K + BK - 1) / BK;
  const int kt0 = blockIdx.z * p.kt_per_split;
  const int kt1 = min(nkt, kt0 + p.kt_per_split);

  const char* Ab;
  if constexpr (AM == CONV_FWD) Ab = (const char*)p.A + (long long)bz * p.sA * 2;
  else Ab = (const char*)p.A + (long long)bz * p.sA * 2 + (AKO ? (long long)m0 * 2 : (long long)m0 * p.lda * 2);
  const char* Bb = (const char*)p.B + (long long)bz * p.sB * 2 + (BKO ? (long long)n0 * 2 : (long long)n0 * p.ldb * 2);
  const long long a_step = AKO ? (long long)BK * p.lda * 2 : BK * 2;
  const long long b_step = BKO ? (long long)BK * p.ldb * 2 : BK * 2;
  const int lim_a = p.M - m0, lim_b = p.N - n0;

  Loader<BM, AM, NW> la;
  Loader<BN, BMD, NW> lb;
  la.init(p, lane, w, p.lda, m0, p.M);
  lb.init(p, lane, w, p.ldb, n0, p.N);
  constexpr int ND = Loader<BM, AM, NW>::NI + Loader<BN, BMD, NW>::NI;  // DMA pieces per wave per K-tile

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto stage = [&](int s) { return smem + s * STAGE; };
  auto issue = [&](int kt, char* stg, bool en) {
    la.issue(p, Ab, a_step, kt, lim_a, stg, w, lane, en);
    lb.issue(p, Bb, b_step, kt, lim_b, stg + A_BYTES, w, lane, en);
  };
  const int ar = wm * TM, bc = wn * TN;
  bf16x8 r0a[FM], r0b[FN], r1a[FM], r1b[FN];
  auto rd = [&](const char* stg, int kk, bf16x8 (&ra)[FM], bf16x8 (&rb)[FN]) {
#pragma unroll
    for (int j = 0; j < FN; ++j) rb[j] = frag<BKO>(stg + A_BYTES, bc + j * 16, kk);
#pragma unroll
    for (int i = 0; i < FM; ++i) ra[i] = frag<AKO>(stg, ar + i * 16, kk);
  };
  auto mm = [&](const bf16x8 (&ra)[FM], const bf16x8 (&rb)[FN]) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rb[j], ra[i], acc[i][j], 0, 0, 0);
  };
  constexpr int NRD = FM * (AKO ? 2 : 1) + FN * (BKO ? 2 : 1);  // ds_read instructions per K-half

  // prologue: tiles kt0 and kt0+1 in flight, wait for kt0, read its k-half 0
  issue(kt0, stage(0), true);
  issue(kt0 + 1, stage(1), kt0 + 1 < kt1);
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(ND) : "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  rd(stage(0), 0, r0a, r0b);

  constexpr int NIA = Loader<BM, AM, NW>::NI;
  // one fragment read (call) of slot q into (ra, rb): B fragments first, then A
  auto rd1 = [&](const char* stg, int kk, int q, bf16x8 (&ra)[FM], bf16x8 (&rb)[FN]) {
    if (q < FN) rb[q] = frag<BKO>(stg + A_BYTES, bc + q * 16, kk);
    else if (q < FN + FM) ra[q - FN] = frag<AKO>(stg, ar + (q - FN) * 16, kk);
  };
  auto mm1 = [&](int q, const bf16x8 (&ra)[FM], const bf16x8 (&rb)[FN]) {
    const int i = q / FN, j = q % FN;
    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rb[j], ra[i], acc[i][j], 0, 0, 0);
  };
  constexpr int NM = FM * FN, NFR = FM + FN;

#pragma unroll 1
  for (int kt = kt0; kt < kt1; ++kt) {
    const int s = (kt - kt0) & 1;
    if constexpr (SCHED == 0) {
      // phase A: MFMAs on k-half 0 || reads of k-half 1
      rd(stage(s), 1, r1a, r1b);
      mm(r0a, r0b);
      interleave<FM * FN, NRD, 0>();
      __builtin_amdgcn_sched_barrier(0);
    } else {
      constexpr int PER = NM / NFR;
#pragma unroll
      for (int q = 0; q < NFR; ++q) {
#pragma unroll
        for (int t = 0; t < PER; ++t) mm1(q * PER + t, r0a, r0b);
        rd1(stage(s), 1, q, r1a, r1b);
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int t = NFR * PER; t < NM; ++t) mm1(t, r0a, r0b);
      __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    // phase B: MFMAs on k-half 1 || DMA of tile kt+2 into the freed stage || reads of tile kt+1's
    // k-half 0 (past the last tile: zero-filling DMA, stale reads -- both unused)
    const bool en = kt + 2 < kt1;
    if constexpr (SCHED == 0) {
      issue(kt + 2, stage(s), en);
      rd(stage(s ^ 1), 0, r0a, r0b);
      mm(r1a, r1b);
      interleave<FM * FN, NRD, ND>();
      __builtin_amdgcn_sched_barrier(0);
    } else {
      // SCHED 1: slot q = {MFMAs, DMA piece q, read q}; SCHED 2: the DMA pieces go to the LAST ND
      // slots and every slot orders its MFMAs first (sched_group_barrier), so the scalar descriptor
      // setup of a piece never sits between the barrier and the first MFMA
      constexpr int SL = NFR > ND ? NFR : ND, PER = NM / SL, D0 = SCHED == 2 ? SL - ND : 0;
#pragma unroll
      for (int q = 0; q < SL; ++q) {
#pragma unroll
        for (int t = 0; t < PER; ++t) mm1(q * PER + t, r1a, r1b);
        const int d = q - D0;
        if (d >= 0 && d < NIA) la.issue(p, Ab, a_step, kt + 2, lim_a, stage(s), w, lane, en, d);
        else if (d >= NIA && d < ND) lb.issue(p, Bb, b_step, kt + 2, lim_b, stage(s) + A_BYTES, w, lane, en, d - NIA);
        rd1(stage(s ^ 1), 0, q, r0a, r0b);
        if constexpr (SCHED == 2) {
          __builtin_amdgcn_sched_group_barrier(0x008, PER, 0);  // the slot's MFMAs first
          __builtin_amdgcn_sched_group_barrier(0x004, 32, 0);   // then its scalar setup
        }
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int t = SL * PER; t < NM; ++t) mm1(t, r1a, r1b);
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (NW == 4) {
      // 256 loop-carried accumulators: pin them to the AGPR half (hipcc 7.2 otherwise carries part
      // of them in VGPRs and shuffles with v_accvgpr moves every iteration)
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) asm volatile("" : "+a"(acc[i][j]));
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
  constexpr int WPS = NW / 4;  // waves per SIMD
  gemm_epilogue<BM, BN, NT, WGM, EPI, (512 / WPS >= 256 ? 4 : 2)>(p, acc, smem, m0, n0, bz);
}

// launch the 8-wave kernel (the 4-wave 128x128-per-wave form runs out of architectural VGPRs for
// its two operand register sets under hipcc 7.2 and shuffles accumulators through v_accvgpr moves
// every K-tile -- not instantiated)
template <int AM, int BMD, int EPI>
int go(int mode, dim3 grid, hipStream_t stream, const GemmParams& p) {
  if (mode == 8) {
    hipLaunchKernelGGL((g5_kernel<AM, BMD, EPI, 2, 4, 0>), grid, dim3(512), 0, stream, p);
    return hipGetLastError() == hipSuccess ? 0 : -2;
  }
  if (mode == 9) {
    hipLaunchKernelGGL((g5_kernel<AM, BMD, EPI, 2, 4, 1>), grid, dim3(512), 0, stream, p);
    return hipGetLastError() == hipSuccess ? 0 : -2;
  }
  if (mode == 10) {
    hipLaunchKernelGGL((g5_kernel<AM, BMD, EPI, 2, 4, 2>), grid, dim3(512), 0, stream, p);
    return hipGetLastError() == hipSuccess ? 0 : -2;
  }
  return -1;
}

}  // namespace g5

// 0: off (default until measured), 8 / 9 / 10: the 8-wave kernel (SCHED 0 / 1 / 2) for every eligible 256x256 GEMM
static int g_g5 = -1;
extern "C" void tfk_g5_set(int waves) { g_g5 = waves; }
static int g5_mode() {
  if (g_g5 < 0) {
    const char* e = getenv("TFK_G5");
    g_g5 = e ? atoi(e) : 0;
  }
  return g_g5;
}

// 256x256 GEMMs: dense fwd (A, B K-inner), dgrad (B K-outer), weight gradients (A, B K-outer, f32
// split-K slabs) and the Cin % 64 == 0 conv-forward gather. -1: not handled here.
extern "C" int tfk_g5_launch(const GemmParams& p_in, int amode, int bmode, int epi, int batch, int splits,
                             hipStream_t stream) {
  const int mode = g5_mode();
  if (mode < 8 || mode > 10) return -1;
  const bool dense = (amode == g4::KIN && (bmode == g4::KIN || bmode == g4::KOUT)) ||
                     (amode == g4::KOUT && bmode == g4::KOUT);
  const bool conv = amode == g4::CONV_FWD && bmode == g4::KIN && (p_in.Cin & 63) == 0;
  if (!dense && !conv) return -1;
  GemmParams p = p_in;
  p.tiles_n = (p.N + g5::BN - 1) / g5::BN;
  const int tiles = ((p.M + g5::BM - 1) / g5::BM) * p.tiles_n;
  const dim3 grid(tiles, batch, splits);
#define TFK_G5(AM_, BMD_, EPI_) \
  if (amode == AM_ && bmode == BMD_ && epi == EPI_) return g5::go<AM_, BMD_, EPI_>(mode, grid, stream, p);
  TFK_G5(g4::KIN, g4::KIN, EPI_BF16)
  TFK_G5(g4::KIN, g4::KIN, EPI_BF16_EXT)
  TFK_G5(g4::KIN, g4::KIN, EPI_F32)
  TFK_G5(g4::KIN, g4::KOUT, EPI_BF16)
  TFK_G5(g4::KIN, g4::KOUT, EPI_BF16_EXT)
  TFK_G5(g4::KIN, g4::KOUT, EPI_BF16_BNR)
  TFK_G5(g4::KOUT, g4::KOUT, EPI_F32)
  TFK_G5(g4::CONV_FWD, g4::KIN, EPI_BF16)
  TFK_G5(g4::CONV_FWD, g4::KIN, EPI_BF16_BNR)
#undef TFK_G5
  return -1;
}

}  // namespace tfk
