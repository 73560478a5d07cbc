// tfk "g4" GEMM engine for gfx950: 4 waves per block (one per SIMD), each wave owning a large
// (BM/2 x BN/2) output tile so that LDS fragment reads per MFMA are halved against 8-wave tiles
// (rocprofv3 on 8192^3: the 8-wave ping-pong kernel issued 1.8x the LDS instructions of
// hipBLASLt's MT256x256x64 4-wave kernel and spent 3.2e8 quad-cycles waiting at barriers;
// profiles/gemm_engine_r2.md). The accumulators live in the AGPR half of the 512-entry register file.
//
// Pipeline per K-tile t (BK = 64, stage s = t & 1, two LDS stages):
//   issue the LDS-DMA of K-tile t+1 into stage s^1        (lands during the whole of tile t)
//   read the k-half-1 fragments of tile t from stage s    (overlaps the k-half-0 MFMAs)
//   MFMAs k-half 0, then k-half 1
//   s_waitcnt vmcnt(0) lgkmcnt(0); barrier               (tile t+1 landed; every read of s retired)
//   read the k-half-0 fragments of tile t+1 from stage s^1
// so HBM/L2 latency hides under one K-tile of MFMAs and each K-tile costs one barrier.
// NST = 3 (one-block-per-CU 8-wave 256x128 / 128x256 tiles, 3 x 48 KiB stages): K-tile t+2 is
// issued at the top of tile t into the stage tile t-1 vacated (its reads retired before the
// barrier that closed t-1), and the end-of-tile wait is the COUNTED s_waitcnt vmcnt(LNI) -- tile
// t+1 landed, tile t+2's LNI DMA instructions per lane still in flight across the raw s_barrier --
// so two K-tiles of MFMAs cover each DMA (cdna_hip_programming.md §5 "Pipelining across barriers").
//
// Operand images (cdna_hip_programming.md §2 T2 / T10; one __shared__ array):
//   K-inner [rows][64 k] bf16, 128-B rows, chunk c of row r at r*128 + ((c ^ (r>>1 & 7)) << 4)
//     -> conflict-free ds_read_b128 row fragments.
//   K-outer blocks of 64 rows: [64 k][64 rows] bf16, chunk c of k-row k at k*128 + ((c ^ swz(k)) << 4),
//     swz(k) = 2*((k>>1 & 1) | (k>>3 & 1)<<1) -> conflict-free ds_read_b64_tr_b16 column fragments.
// LDS-DMA writes 1 KiB lane-linear per wave instruction (8 image rows / 8 k-rows, full 128-B
// global lines), so the swizzle goes on the per-lane SOURCE address (rule 21). Out-of-range
// rows/k read zeros: the buffer descriptor range check returns 0 for offsets past num_records.
//
// Operand modes: A_KIN / A_KOUT / A_CONV_FWD (implicit-GEMM gather, Cin % 64 == 0: a K-tile is one
// (r,s) tap and 64 channels; Cin % 8 == 0 below 64: 64/Cin taps per K-tile) x B_KIN / B_KOUT / B_CONV_WGRAD (im2col of X as the K-outer operand of
// a weight gradient: GEMM k = output pixel (n,p,q), column = (r,s,c); each lane's 16-B chunk is 8
// channels of one tap, so C % 8 == 0; the pixel of a K-tile row is found with magic-number
// division). Epilogues: gemm_epilogue.h (LDS-staged).
#include "common.h"
#include <algorithm>
#include "gemm_params.h"
#include "gemm_epilogue.h"
#include "g4_loader.h"

namespace tfk {
namespace g4 {

// Block = (BM/64) x (BN/64) waves, each owning a 64x64 output tile (4x4 16x16 fragments): the
// 128x128 tile runs 4 waves at two blocks per CU, 256x128 runs 8 and 256x256 runs 16 waves (one
// block per CU, 128 KiB of stages) -- occupancy from co-resident waves, not one big wave per SIMD
// (measured: 1-wave/SIMD 128x128 wave tiles spill AGPR accumulators under hipcc 7.2).
template <int BM, int BN>
constexpr int nwaves() { return (BM / 64) * (BN / 64); }

// OCC = 4: short-K variant for blocks that own exactly ONE K-tile (K <= 64 per split: the 1x1
// convs of ResNet stage 2, M=802816 x N=256 x K=64). Such a block is load -> 32 MFMAs -> epilogue
// with nothing to pipeline, so latency is hidden by co-resident blocks instead: one LDS stage
// (36 KiB with the epilogue image) and <= 128 VGPRs put 4 blocks (16 waves) on a CU instead of 2.
template <int BM, int BN>
constexpr int occ_default() { return (BM * BN <= 128 * 128) ? 2 : 1; }

template <int BM, int BN, int AM, int BMD, int EPI, int OCC = occ_default<BM, BN>(), int NST = 2>
__global__ __launch_bounds__((nwaves<BM, BN>() * 64), OCC) void g4_kernel(GemmParams p) {
  constexpr int NW = nwaves<BM, BN>(), NTH = NW * 64, WGM = BM / 64, WGN = BN / 64;
  constexpr int LBM = BMD == 2 ? CONV_WGRAD : BMD;  // B_CONV_WGRAD (= 2 in the B-mode numbering)
  constexpr bool AKO = (AM == KOUT), BKO = (LBM == KOUT || LBM == CONV_WGRAD);
  constexpr int WTM = 64, WTN = 64, FM = 4, FN = 4;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE = A_BYTES + B_BYTES;
  // SHORTK: one LDS stage, no intra-block double buffering (the host launches it for blocks of
  // <= g_shortk K-tiles); co-resident blocks hide the DMA latency instead
  constexpr bool SHORTK = OCC > occ_default<BM, BN>();
  static_assert(NST == 2 || (NST == 3 && !SHORTK), "stages: 2, or 3 without SHORTK");
  constexpr int MAIN = (SHORTK ? 1 : NST) * STAGE, EPIB = epi_lds_bytes<BM, BN, WGM>();
  __shared__ __attribute__((aligned(16))) char smem[MAIN > EPIB ? MAIN : EPIB];

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w / WGN, wn = w % WGN;
  const int bz = blockIdx.y;

  // tile order: XCD remap, then GROUP_M = 4 inside each XCD's contiguous range
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
  const char* Bb = (const char*)p.B + (long long)bz * p.sB * 2 +
                   (LBM == CONV_WGRAD ? 0LL : BKO ? (long long)n0 * 2 : (long long)n0 * p.ldb * 2);
  const long long a_step = AKO ? (long long)BK * p.lda * 2 : BK * 2;
  const long long b_step = BKO ? (long long)BK * p.ldb * 2 : BK * 2;
  const int lim_a = p.M - m0, lim_b = p.N - n0;

  Loader<BM, AM, NW, !SHORTK> la;
  Loader<BN, LBM, NW> lb;
  la.init(p, lane, w, p.lda, m0, p.M);
  lb.init(p, lane, w, p.ldb, n0, p.N);

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto stage_ptr = [&](int s) { return smem + s * STAGE; };

  // DMA instructions per lane per K-tile (the counted wait of the 3-stage pipeline)
  constexpr int LNI = Loader<BM, AM, NW, !SHORTK>::NI + Loader<BN, LBM, NW>::NI;
  static_assert(LNI <= 60, "vmcnt field");
  la.issue(p, Ab, a_step, kt0, lim_a, stage_ptr(0), w, lane);
  lb.issue(p, Bb, b_step, kt0, lim_b, stage_ptr(0) + A_BYTES, w, lane);
  if constexpr (NST == 3) {
    if (kt0 + 1 < kt1) {
      la.issue(p, Ab, a_step, kt0 + 1, lim_a, stage_ptr(1), w, lane);
      lb.issue(p, Bb, b_step, kt0 + 1, lim_b, stage_ptr(1) + A_BYTES, w, lane);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LNI) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  // B fragments of a K-half are held for the whole half (FN x 4 VGPRs); A fragments stream, one
  // 16-row fragment at a time (read one ahead of its FN MFMAs), so the double-buffered operand
  // registers stay at 2*FN*4 + ~3*4 next to the AGPR accumulators.
  bf16x8 b0[FN], b1[FN];
  const int ar = wm * WTM, bc = wn * WTN;
  {
    const char* As = stage_ptr(0);
#pragma unroll
    for (int j = 0; j < FN; ++j) b0[j] = frag<BKO>(As + A_BYTES, bc + j * 16, 0);
  }

  int s3 = 0;  // NST = 3: stage of tile kt (kt - kt0) % 3, carried without a division
#pragma unroll 1
  for (int kt = kt0; kt < kt1; ++kt) {
    const int s = NST == 3 ? s3 : SHORTK ? 0 : (kt - kt0) & 1;
    const char* As = stage_ptr(s);
    const char* Bs = As + A_BYTES;
    const bool more = kt + 1 < kt1;
    if constexpr (NST == 3) {
      if (kt + 2 < kt1) {
        char* nx = stage_ptr(s == 0 ? 2 : s - 1);  // = (s + 2) % 3: tile kt-1's stage
        la.issue(p, Ab, a_step, kt + 2, lim_a, nx, w, lane);
        lb.issue(p, Bb, b_step, kt + 2, lim_b, nx + A_BYTES, w, lane);
      }
    } else if (!SHORTK && more) {
      char* nx = stage_ptr(s ^ 1);
      la.issue(p, Ab, a_step, kt + 1, lim_a, nx, w, lane);
      lb.issue(p, Bb, b_step, kt + 1, lim_b, nx + A_BYTES, w, lane);
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) b1[j] = frag<BKO>(Bs, bc + j * 16, 1);
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const bf16x8 a = frag<AKO>(As, ar + i * 16, 0);
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b0[j], a, acc[i][j], 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const bf16x8 a = frag<AKO>(As, ar + i * 16, 1);
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b1[j], a, acc[i][j], 0, 0, 0);
    }
    if (more) {
      if constexpr (SHORTK) {
        // every wave's reads of the single stage are done before the next K-tile overwrites it
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        la.issue(p, Ab, a_step, kt + 1, lim_a, stage_ptr(0), w, lane);
        lb.issue(p, Bb, b_step, kt + 1, lim_b, stage_ptr(0) + A_BYTES, w, lane);
      }
      int nxs;
      if constexpr (NST == 3) {
        nxs = s == 2 ? 0 : s + 1;
        s3 = nxs;
        if (kt + 2 < kt1)
          asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(LNI) : "memory");  // tile kt+1 landed
        else
          asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      } else {
        nxs = SHORTK ? 0 : s ^ 1;
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      const char* Bn = stage_ptr(nxs) + A_BYTES;
#pragma unroll
      for (int j = 0; j < FN; ++j) b0[j] = frag<BKO>(Bn, bc + j * 16, 0);
    }
  }
  __syncthreads();
  // BN-reduce chunks in flight per thread by VGPR budget: 512 / (waves per SIMD); 3 at 4 waves per
  // SIMD (2 measured 20.49 ms/step ResNet-50, 3 20.44 -- spill-free since the activation-free epilogue)
  constexpr int WPS = (NW * OCC) / 4 > 0 ? (NW * OCC) / 4 : 1;
  gemm_epilogue<BM, BN, NTH, WGM, EPI, (512 / WPS >= 256 ? 4 : 3)>(p, acc, smem, m0, n0, bz);
}

// ---------------------------------------------------------------------------------------------
// MX-fp8 on the g4 engine: A [M][K] and B [N][K] e4m3 bytes (both K-inner), e8m0 scales [rows][K/32].
// A K-tile is 128 fp8 bytes per row -- byte-for-byte the 128-B row image of a bf16 BK=64 tile, so
// the LDS-DMA Loader and the XOR-swizzled image are reused unchanged (driven with bf16-equivalent
// strides: K/2, ld/2). One v_mfma_scale_f32_16x16x128_f8f6f4 consumes a whole K-tile row pair
// (lane (row l&15, group g = l>>4) holds 16-B chunks g and g+4 = the two K-halves of the bf16
// fragment reader), at twice the bf16 MFMA rate. The 4 scale bytes of a row's K-tile are one u32,
// loaded from global one tile ahead (L2-resident, 4 B per row per 128 K) into registers; lane group
// g uses byte g. 4-wave 128x128 blocks (64x64 wave tiles), 2 LDS stages, shared epilogue.
template <int BM, int BN, int EPI>
__global__ __launch_bounds__((nwaves<BM, BN>() * 64), (occ_default<BM, BN>())) void g4_fp8_kernel(GemmParams p,
                                                                                               int sld) {
  constexpr int NW = nwaves<BM, BN>(), NTH = NW * 64, WGM = BM / 64, WGN = BN / 64;
  constexpr int FM = 4, FN = 4;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  // + the K-tile's scale words of every A and B row ([BM] + [BN] u32), DMA'd with the operands
  constexpr int SA_OFF = A_BYTES + B_BYTES, SB_OFF = SA_OFF + BM * 4, STAGE = SB_OFF + BN * 4;
  constexpr int MAIN = 2 * STAGE, EPIB = epi_lds_bytes<BM, BN, WGM>();
  __shared__ __attribute__((aligned(16))) char smem[MAIN > EPIB ? MAIN : EPIB];

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w / WGN, wn = w % WGN;
  const int tiles_m = (p.M + BM - 1) / BM;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  constexpr int GM = 4;
  const int grp = tile / (GM * p.tiles_n), first_m = grp * GM;
  const int gm = min(GM, tiles_m - first_m), inr = tile - grp * GM * p.tiles_n;
  const int m0 = (first_m + inr % gm) * BM, n0 = (inr / gm) * BN;
  // p.K / p.lda / p.ldb arrive in bf16-equivalent units (bytes / 2): the Loader's byte math holds
  const int nkt = (p.K + BK - 1) / BK;
  const int kt0 = blockIdx.z * p.kt_per_split;
  const int kt1 = min(nkt, kt0 + p.kt_per_split);
  const char* Ab = (const char*)p.A + (long long)m0 * p.lda * 2;
  const char* Bb = (const char*)p.B + (long long)n0 * p.ldb * 2;
  const int lim_a = p.M - m0, lim_b = p.N - n0;
  Loader<BM, KIN, NW> la;
  Loader<BN, KIN, NW> lb;
  la.init(p, lane, w, p.lda, m0, p.M);
  lb.init(p, lane, w, p.ldb, n0, p.N);

  // Scales: the K-tile's 4 scale bytes of each row (one u32) go to LDS by LDS-DMA next to the
  // operands (buffer_load_dword ... lds: 64 rows per instruction, lane-linear; rows past M/N are
  // past num_records -> 0 and multiply zero-filled operands); waves 0 .. BM/64 + BN/64 - 1 issue
  // one instruction each. Lane group g of a fragment then reads byte g of its row's word.
  const int g = lane >> 4, li = lane & 15;
  constexpr int SCA_I = BM / 64, SC_I = BM / 64 + BN / 64;
  static_assert(SC_I <= NW, "one scale DMA per wave");
  const bool sc_issuer = w < SC_I;  // wave-uniform
  const bool sc_is_a = w < SCA_I;
  const int sc_row = (sc_is_a ? m0 + w * 64 : n0 + (w - SCA_I) * 64) + lane;
  const int sc_img = sc_is_a ? SA_OFF + w * 256 : SB_OFF + (w - SCA_I) * 256;
  const __amdgpu_buffer_rsrc_t rsc = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(sc_is_a ? p.a_scale : p.b_scale), (short)0,
      (int)min((long long)(sc_is_a ? p.M : p.N) * sld, (long long)NREC), 0x00020000);
  auto issue_scales = [&](int kt, char* stg) {
    if (sc_issuer)
      lds_dma<4>(rsc, (LDS_AS void*)(stg + sc_img), sc_row * sld + kt * 4);
  };
  auto read_scales = [&](const char* stg, int (&sa)[FM], int (&sb)[FN]) {
#pragma unroll
    for (int i = 0; i < FM; ++i) sa[i] = *(const unsigned char*)(stg + SA_OFF + (wm * 64 + i * 16 + li) * 4 + g);
#pragma unroll
    for (int j = 0; j < FN; ++j) sb[j] = *(const unsigned char*)(stg + SB_OFF + (wn * 64 + j * 16 + li) * 4 + g);
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto stage_ptr = [&](int st) { return smem + st * STAGE; };
  if (kt0 < kt1) {
    la.issue(p, Ab, BK * 2, kt0, lim_a, stage_ptr(0), w, lane);
    lb.issue(p, Bb, BK * 2, kt0, lim_b, stage_ptr(0) + A_BYTES, w, lane);
    issue_scales(kt0, stage_ptr(0));
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  const int ar = wm * 64, bc = wn * 64;

#pragma unroll 1
  for (int kt = kt0; kt < kt1; ++kt) {
    const int st = (kt - kt0) & 1;
    const char* As = stage_ptr(st);
    const char* Bs = As + A_BYTES;
    const bool more = kt + 1 < kt1;
    if (more) {
      char* nx = stage_ptr(st ^ 1);
      la.issue(p, Ab, BK * 2, kt + 1, lim_a, nx, w, lane);
      lb.issue(p, Bb, BK * 2, kt + 1, lim_b, nx + A_BYTES, w, lane);
      issue_scales(kt + 1, nx);
    }
    int sa[FM], sb[FN];
    read_scales(As, sa, sb);
    i32x8 bfr[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const bf16x8 lo = frag<false>(Bs, bc + j * 16, 0), hi = frag<false>(Bs, bc + j * 16, 1);
      bfr[j] = pack8(lo, hi);
    }
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const bf16x8 lo = frag<false>(As, ar + i * 16, 0), hi = frag<false>(As, ar + i * 16, 1);
      const i32x8 a = pack8(lo, hi);
#pragma unroll
      for (int j = 0; j < FN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(bfr[j], a, acc[i][j], 0, 0, 0, sb[j], 0, sa[i]);
    }
    if (more) {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
  }
  __syncthreads();
  gemm_epilogue<BM, BN, NTH, WGM, EPI>(p, acc, smem, m0, n0, 0);
}

}  // namespace g4
}  // namespace tfk

using namespace tfk;

// Eligibility: 16-B aligned operand rows, K % 8 == 0 (a chunk never straddles K), K-outer row
// counts % 8 == 0; conv gather: Cin % 64 == 0 (a K-tile = one tap x 64 channels).
extern "C" int tfk_g4_ok(const GemmParams& p, int amode, int bmode) {
  if (!(amode == 0 || amode == 1 || amode == 2) || bmode > 2) return 0;
  if (bmode == 2 && ((p.Cin & 7) || amode != 1 || (long long)p.Nimg * p.H * p.W * p.Cin >= (1LL << 30) ||
                     (long long)p.Nimg * p.P * p.Q >= (1LL << 31) - 64)) return 0;
  if ((p.K & 7) || (p.ldb & 7)) return 0;
  if (amode != 2 && (p.lda & 7)) return 0;
  if (((uintptr_t)p.A & 15) || ((uintptr_t)p.B & 15)) return 0;
  if ((p.sA & 7) || (p.sB & 7)) return 0;
  if (amode == 1 && (p.M & 7)) return 0;
  if (bmode >= 1 && (p.N & 7)) return 0;
  // conv-fwd gather: Cin % 64 == 0 (one tap per K-tile) or Cin % 8 == 0 below 64 (taps per K-tile)
  if (amode == 2 && (((p.Cin & 63) && ((p.Cin & 7) || p.Cin > 64)) || (long long)p.Nimg * p.H * p.W * p.Cin >= (1LL << 30)))
    return 0;
  return 1;
}

#define TFK_G4_CASE(BM_, BN_, AM_, BM2_, EPI_)                                                      \
  if (bm == BM_ && bn == BN_ && amode == AM_ && bmode == BM2_ && epi == EPI_) {                     \
    hipLaunchKernelGGL((g4::g4_kernel<BM_, BN_, AM_, BM2_, EPI_>), dim3(tiles, batch, splits),                \
                       dim3(g4::nwaves<BM_, BN_>() * 64), 0,                                           \
                       stream, p);                                                                  \
    return hipGetLastError() == hipSuccess ? 0 : -2;                                                \
  }
#define TFK_G4_TILES(AM_, BM2_, EPI_) TFK_G4_CASE(256, 256, AM_, BM2_, EPI_) TFK_G4_CASE(128, 128, AM_, BM2_, EPI_)
// 2-wave tiles for 64-wide operands (Cout = 64 weight gradients, 64-channel dgrads)
#define TFK_G4_NARROW(AM_, BM2_, EPI_) TFK_G4_CASE(128, 64, AM_, BM2_, EPI_) TFK_G4_CASE(64, 128, AM_, BM2_, EPI_)

// 8-wave one-block-per-CU tiles with the 3-stage LDS ring (NST = 3)
#define TFK_G4_DEEP_CASE(BM_, BN_, AM_, BM2_, EPI_)                                                  \
  if (bm == BM_ && bn == BN_ && amode == AM_ && bmode == BM2_ && epi == EPI_) {                     \
    hipLaunchKernelGGL((g4::g4_kernel<BM_, BN_, AM_, BM2_, EPI_, 1, 3>), dim3(tiles, batch, splits),  \
                       dim3(g4::nwaves<BM_, BN_>() * 64), 0, stream, p);                            \
    return hipGetLastError() == hipSuccess ? 0 : -2;                                                \
  }
#define TFK_G4_DEEP(AM_, BM2_, EPI_) TFK_G4_DEEP_CASE(256, 128, AM_, BM2_, EPI_) TFK_G4_DEEP_CASE(128, 256, AM_, BM2_, EPI_)

#define TFK_G4_SHORTK(AM_, BM2_, EPI_)                                                               \
  if (amode == AM_ && bmode == BM2_ && epi == EPI_) {                                               \
    hipLaunchKernelGGL((g4::g4_kernel<128, 128, AM_, BM2_, EPI_, 4>), dim3(tiles, batch, splits),    \
                       dim3(g4::nwaves<128, 128>() * 64), 0, stream, p);                            \
    return hipGetLastError() == hipSuccess ? 0 : -2;                                                \
  }

#ifndef G4_SHORTK_DEFAULT_KT
#define G4_SHORTK_DEFAULT_KT 8  // measured ResNet-50 bs256: 2 -> 27.42, 4 -> 27.04, 8 -> 26.71, 16 -> 26.67 ms
#endif
// Max K-tiles per block for the single-stage 4-blocks-per-CU 128x128 variant (0 = off).
// TFK_G4_SHORTK=<n> overrides the default.
static int g_shortk = -1;
static int shortk_max_kt() {
  if (g_shortk < 0) {
    const char* e = getenv("TFK_G4_SHORTK");
    g_shortk = e ? atoi(e) : G4_SHORTK_DEFAULT_KT;
  }
  return g_shortk;
}
// < 0: back to the environment / built-in default
extern "C" void tfk_g4_set_shortk(int max_kt) { g_shortk = max_kt < 0 ? -1 : max_kt; }

static void fast_div(unsigned d, unsigned* mul, int* shift) {
  int s = 0;
  while ((1ull << s) < d) ++s;
  *shift = s;
  *mul = (unsigned)(((1ull << 32) * ((1ull << s) - d)) / d + 1);
}

// p.tiles_n / p.kt_per_split set by the caller (tfk_gemm_launch). Returns -1 if not instantiated.
extern "C" int tfk_halo_launch(const GemmParams& p, int epi, int batch, int splits, hipStream_t stream);
extern "C" int tfk_g8_launch(const GemmParams& p, int amode, int bmode, int epi, int batch, int splits,
                             hipStream_t stream);
extern "C" int tfk_g5_launch(const GemmParams& p, int amode, int bmode, int epi, int batch, int splits,
                             hipStream_t stream);

extern "C" int tfk_g4_launch(const GemmParams& p_in, int bm, int bn, int amode, int bmode, int epi, int batch,
                             int splits, hipStream_t stream) {
  // 3x3 / stride-1 convs of the supported shapes: the halo-tile direct conv (conv_halo.hip)
  if (amode == 2 && bmode == 0) {
    const int r = tfk_halo_launch(p_in, epi, batch, splits, stream);
    if (r != -1) return r;
  }
  // 256x256: the mid-tile-barrier engine (gemm_g5.hip) or the 8-phase engine (gemm_g8.hip) when enabled
  if (bm == 256 && bn == 256) {
    int r = tfk_g5_launch(p_in, amode, bmode, epi, batch, splits, stream);
    if (r != -1) return r;
    r = tfk_g8_launch(p_in, amode, bmode, epi, batch, splits, stream);
    if (r != -1) return r;
  }
  GemmParams p = p_in;
  p.tiles_n = (p.N + bn - 1) / bn;
  const int tiles = ((p.M + bm - 1) / bm) * p.tiles_n;
  if (bmode == 2) {
    fast_div((unsigned)p.Q, &p.fd_q_mul, &p.fd_q_shift);
    fast_div((unsigned)(p.P * p.Q), &p.fd_pq_mul, &p.fd_pq_shift);
  }
  if (amode == 2 && p.Cin < 64) {
    fast_div((unsigned)p.S, &p.fd_q_mul, &p.fd_q_shift);
    fast_div((unsigned)p.Cin, &p.fd_pq_mul, &p.fd_pq_shift);
  }
  // few K-tiles per block: the 4-blocks-per-CU single-stage instantiations (TFK_G4_SHORTK=0: off;
  // one K-tile measured ResNet-50 bs256: 30.40 -> 29.72 ms/step)
  if (p.kt_per_split <= shortk_max_kt() && bm == 128 && bn == 128 && !(amode == 2 && p.Cin < 64)) {
    TFK_G4_SHORTK(0, 0, EPI_BF16)
    TFK_G4_SHORTK(0, 1, EPI_BF16)
    TFK_G4_SHORTK(0, 1, EPI_BF16_BNR)
    TFK_G4_SHORTK(2, 0, EPI_BF16)
    TFK_G4_SHORTK(2, 0, EPI_BF16_BNR)
  }
  TFK_G4_DEEP(0, 0, EPI_BF16)
  TFK_G4_DEEP(0, 0, EPI_BF16_EXT)
  TFK_G4_DEEP(0, 1, EPI_BF16)
  TFK_G4_DEEP(0, 1, EPI_BF16_EXT)
  TFK_G4_DEEP(0, 1, EPI_BF16_BNR)
  TFK_G4_DEEP(1, 1, EPI_F32)
  TFK_G4_DEEP(2, 0, EPI_BF16)
  TFK_G4_DEEP(2, 0, EPI_BF16_BNR)
  TFK_G4_DEEP(1, 2, EPI_F32)
  TFK_G4_TILES(0, 0, EPI_BF16)
  TFK_G4_TILES(0, 0, EPI_F32)
  TFK_G4_TILES(0, 0, EPI_BF16_EXT)
  TFK_G4_TILES(0, 1, EPI_BF16)
  TFK_G4_TILES(0, 1, EPI_F32)
  TFK_G4_TILES(0, 1, EPI_BF16_EXT)
  TFK_G4_TILES(0, 1, EPI_BF16_BNR)
  TFK_G4_TILES(1, 1, EPI_F32)
  TFK_G4_TILES(1, 1, EPI_BF16)
  TFK_G4_TILES(2, 0, EPI_BF16)
  TFK_G4_TILES(0, 0, EPI_BF16_ACT)  // activated bf16 outputs (EPI_BF16's epilogue is activation-free)
  TFK_G4_TILES(2, 0, EPI_BF16_ACT)
  // stride-1 conv dgrad run as a forward conv over dY with flipped weights (ops/gemm.py), carrying
  // the fused BN-backward reduction of the layer that produced x
  TFK_G4_TILES(2, 0, EPI_BF16_BNR)
  // weight gradients with one narrow side (Cout or Cin = 64..256 of a huge-K 1x1 conv): 4-wave
  // 64x256 / 256x64 blocks -- every wave a full 64x64 MFMA tile, no zero-filled half of a 128x128
  TFK_G4_CASE(64, 256, 1, 1, EPI_F32)
  TFK_G4_CASE(256, 64, 1, 1, EPI_F32)
  // conv weight gradients: dY (K-outer) x im2col(X) gather, f32 split-K slabs
  TFK_G4_TILES(1, 2, EPI_F32)
  TFK_G4_NARROW(1, 2, EPI_F32)
  TFK_G4_NARROW(2, 0, EPI_BF16_BNR)
  TFK_G4_NARROW(2, 0, EPI_BF16)
  // 64-channel 3x3 convs (ResNet stage 1): 4-wave 256x64 blocks, the 64-wide B tile shared by 256
  // gathered rows (forward, and the stride-1 dgrad as a forward conv with the BN-reduce epilogue)
  TFK_G4_CASE(256, 64, 2, 0, EPI_BF16)
  TFK_G4_CASE(256, 64, 2, 0, EPI_BF16_BNR)
  TFK_G4_NARROW(0, 1, EPI_BF16_BNR)
  TFK_G4_NARROW(0, 1, EPI_F32)
  TFK_G4_NARROW(1, 1, EPI_F32)
  TFK_G4_NARROW(0, 0, EPI_BF16)
  TFK_G4_NARROW(0, 1, EPI_BF16)
  return -1;
}

// MX-fp8 GEMM on the g4 engine. p in BYTES (K, lda, ldb = bytes per row); needs K % 128 == 0,
// lda/ldb % 16 == 0 and 16-B aligned operands. Returns -1 when not eligible (caller falls back).
// Tile of the fp8 engine: 0 = by shape (256x256 16-wave blocks when they fill the chip, else
// 128x128), 128 / 256 / 2561 (= 256x128, 8 waves) forced
// (TFK_FP8_TILE or tfk_fp8_set_tile).
static int g_fp8_tile = -1;
extern "C" void tfk_fp8_set_tile(int t) { g_fp8_tile = t; }
extern "C" int tfk_g4_fp8_launch(const GemmParams& p_in, int epi, int splits, hipStream_t stream) {
  GemmParams p = p_in;
  if ((p.K & 127) || (p.lda & 15) || (p.ldb & 15) || (((uintptr_t)p.A | (uintptr_t)p.B) & 15) ||
      (((uintptr_t)p.a_scale | (uintptr_t)p.b_scale) & 3))
    return -1;
  if (g_fp8_tile < 0) {
    const char* e = getenv("TFK_FP8_TILE");
    g_fp8_tile = e ? atoi(e) : 0;
  }
  if (epi == EPI_BF16_EXT_MX &&
      (splits > 1 || (p.M & 31) || (p.N & 31) || p.ldc != p.N || !p.mx_qr || !p.mx_sr || !p.mx_qc || !p.mx_sc))
    return -2;
  const int sld = p.K / 32;
  p.K /= 2;
  p.lda /= 2;
  p.ldb /= 2;
  const int nkt = (p.K + g4::BK - 1) / g4::BK;
  const long long t256 = (long long)((p.M + 255) / 256) * ((p.N + 255) / 256);
  if (splits < 1) splits = 1;
  if (splits > nkt) splits = nkt;
  p.kt_per_split = (nkt + splits - 1) / splits;
  splits = (nkt + p.kt_per_split - 1) / p.kt_per_split;
  const bool big = g_fp8_tile == 256 || (g_fp8_tile == 0 && p.M >= 256 && p.N >= 256 && t256 * splits >= 240);
  // 256x128 (8 waves of 64x64, one block per CU), forced only (2561): on the few-tile Transformer-big
  // shapes 256x256 cannot fill ([8192][1024] dgrads: 128 tiles of 256x256, 256 of 256x128) it
  // measured slower than two 128x128 blocks per CU (43.9 vs 38.9 us per dgrad, 47.0 vs 41.1 per
  // EXT forward; profiles/perf_log_r5.md), so the shape rule keeps 128x128 there
  const bool rect = !big && g_fp8_tile == 2561;
  const int TM = big || rect ? 256 : 128, TN = big ? 256 : 128;
  p.tiles_n = (p.N + TN - 1) / TN;
  const int tiles = ((p.M + TM - 1) / TM) * p.tiles_n;
  if (p.stats_shards < 1) p.stats_shards = 1;
  const dim3 grid(tiles, 1, splits);
#define TFK_FP8_G4(BTM, BTN)                                                                                    \
  {                                                                                                             \
    const dim3 block(g4::nwaves<BTM, BTN>() * 64);                                                              \
    if (epi == EPI_F32)                                                                                         \
      hipLaunchKernelGGL((g4::g4_fp8_kernel<BTM, BTN, EPI_F32>), grid, block, 0, stream, p, sld);               \
    else if (epi == EPI_BF16_EXT)                                                                               \
      hipLaunchKernelGGL((g4::g4_fp8_kernel<BTM, BTN, EPI_BF16_EXT>), grid, block, 0, stream, p, sld);          \
    else if (epi == EPI_BF16_EXT_MX)                                                                            \
      hipLaunchKernelGGL((g4::g4_fp8_kernel<BTM, BTN, EPI_BF16_EXT_MX>), grid, block, 0, stream, p, sld);       \
    else                                                                                                        \
      hipLaunchKernelGGL((g4::g4_fp8_kernel<BTM, BTN, EPI_BF16>), grid, block, 0, stream, p, sld);              \
  }
  if (big) {
    TFK_FP8_G4(256, 256)
  } else if (rect) {
    TFK_FP8_G4(256, 128)
  } else {
    TFK_FP8_G4(128, 128)
  }
#undef TFK_FP8_G4
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
