// tfk "g8" GEMM engine for gfx950: 256x256 output tile, 8 waves (2 x 4), BK = 64, the 8-phase
// schedule of cdna_hip_programming.md §5 "The 256² 8-phase template" written for this codebase's
// LDS-DMA loaders and XOR-swizzled operand images (g4_loader.h) and its shared epilogue.
//
// Wave (wr, wc) owns four 64x32 quadrant sub-tiles: rows {qm*128 + wr*64 + [0,64)} x cols
// {qn*128 + wc*32 + [0,32)}, qm, qn in {0,1} -- so quadrant (qm, qn) reads only A half qm (rows
// qm*128..+127) and B half qn of a K-tile. Each K-tile is staged as four 16-KiB half-images
// (A0, A1, B0, B1; 2 LDS-DMA instructions per lane each) in one of two 64-KiB buffers (tile t in
// buffer t & 1: 128 KiB). A K-tile is computed in 4 phases, one quadrant each (16 MFMA 16x16x32 per
// wave): Q(0,0) reads A0 + B0, Q(0,1) B1, Q(1,1) A1, Q(1,0) B0 again (register budget). Every
// phase: its fragment ds_reads, ONE half-image DMA, barrier, lgkmcnt(0), setprio(1), 16 MFMAs,
// setprio(0), barrier. The half-image a phase restages is the one whose last reads retired before
// the previous phase's closing barrier:
//   phase 0 of tile u: B0(u+1) -> buffer (u+1)&1   (B0(u-1) last read in phase 3 of u-1)
//   phase 1:           A0(u+2) -> buffer u&1       (A0(u) read in phase 0)
//   phase 2:           B1(u+2)                     (B1(u) read in phase 1)
//   phase 3:           A1(u+2)                     (A1(u) read in phase 2)
// so ~1.5 K-tiles of DMA are in flight; phase 3 ends with the COUNTED s_waitcnt vmcnt(6) (tile
// u+1's four halves landed, the three halves issued since stay in flight across the raw barrier)
// and tile u+1 is read from the next phase on ("read a staged buffer one phase after the wait
// that retires it").
//
// Ping-pong: the two wave groups (wr = 0: waves 0-3, wr = 1: waves 4-7) run ONE BARRIER APART --
// group 1 passes an extra barrier before the loop, group 0 one after it -- so each barrier pairs
// group 0's "MFMAs done" with group 1's "fragments read", and one group's 16-MFMA cluster runs
// while the other issues its ds_reads and DMA. Under the stagger a wave may pass the barrier that
// closes phase p-1 while the other group has only ISSUED its phase p-1 reads, so each phase retires
// its own ds_reads (lgkmcnt(0)) BEFORE its first barrier: a half-image restaged in phase p (one
// phase after its last read) is then never overwritten under an in-flight read.
// (Lockstep form, no stagger: 1046 / 999 TF/s sq4096 fwd / dgrad vs the g4 256x256 tile's
// 1217 / 1156, profiles/tile_ab_r4b.jsonl.)
#include "common.h"
#include "gemm_params.h"
#include "gemm_epilogue.h"
#include "g4_loader.h"

namespace tfk {
namespace g8 {

using g4::BK;
using g4::CONV_FWD;
using g4::frag;
using g4::KIN;
using g4::KOUT;
using g4::Loader;

constexpr int BM = 256, BN = 256, NW = 8, NT = 512, HALF = 128;
constexpr int HBYTES = HALF * BK * 2;  // 16 KiB half-image
constexpr int BUF = 4 * HBYTES;        // A0, A1, B0, B1
enum { A0 = 0, A1 = 1, B0 = 2, B1 = 3 };

__device__ __forceinline__ void bar() {
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// AM: KIN (dense A [M][K]), KOUT (dense A stored [K][M]: weight gradients dY^T X) or CONV_FWD
// (implicit-GEMM gather of NHWC x, Cin % 64 == 0: a K-tile is one (r, s) tap x 64 channels);
// BMD: KIN or KOUT.
template <int AM, int BMD, int EPI>
__global__ __launch_bounds__(NT, 1) void g8_kernel(GemmParams p) {
  constexpr bool AKO = (AM == KOUT), BKO = (BMD == KOUT);
  constexpr int MAIN = 2 * BUF, EPIB = epi_lds_bytes<BM, BN, 2>();
  __shared__ __attribute__((aligned(16))) char smem[MAIN > EPIB ? MAIN : EPIB];

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 2, wc = w & 3;
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

  // one loader per half-image (its rows are the half's 128 rows)
  const char* Abase = (const char*)p.A + (long long)bz * p.sA * 2;
  const char* Bbase = (const char*)p.B + (long long)bz * p.sB * 2;
  const char* Ah[2] = {AM == CONV_FWD ? Abase : Abase + (AKO ? (long long)m0 * 2 : (long long)m0 * p.lda * 2),
                       AM == CONV_FWD ? Abase
                                      : Abase + (AKO ? (long long)(m0 + HALF) * 2 : (long long)(m0 + HALF) * p.lda * 2)};
  const char* Bh[2] = {Bbase + (BKO ? (long long)n0 * 2 : (long long)n0 * p.ldb * 2),
                       Bbase + (BKO ? (long long)(n0 + HALF) * 2 : (long long)(n0 + HALF) * p.ldb * 2)};
  const long long a_step = AKO ? (long long)BK * p.lda * 2 : BK * 2;
  const long long b_step = BKO ? (long long)BK * p.ldb * 2 : BK * 2;
  const int lim_a[2] = {p.M - m0, p.M - m0 - HALF};
  const int lim_b[2] = {p.N - n0, p.N - n0 - HALF};
  Loader<HALF, AM, NW, false> la0, la1;
  Loader<HALF, BMD, NW> lb0, lb1;
  la0.init(p, lane, w, p.lda, m0, p.M);
  la1.init(p, lane, w, p.lda, m0 + HALF, p.M);
  lb0.init(p, lane, w, p.ldb, n0, p.N);
  lb1.init(p, lane, w, p.ldb, n0 + HALF, p.N);
  auto himg = [&](int buf, int h) { return smem + buf * BUF + h * HBYTES; };
  auto issue = [&](int h, int kt) {  // half-image h of K-tile kt into buffer kt & 1
    char* img = himg(kt & 1, h);
    if (h == A0) la0.issue(p, Ah[0], a_step, kt, lim_a[0], img, w, lane);
    else if (h == A1) la1.issue(p, Ah[1], a_step, kt, lim_a[1], img, w, lane);
    else if (h == B0) lb0.issue(p, Bh[0], b_step, kt, lim_b[0], img, w, lane);
    else lb1.issue(p, Bh[1], b_step, kt, lim_b[1], img, w, lane);
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue, in the steady state's issue order: A0 B1 A1 (phases 1-3 of tile kt0-2), B0 (phase 0
  // of kt0-1), then A0 B1 A1 of kt0+1 (phases 1-3 of kt0-1)
  if (kt0 < kt1) {
    issue(A0, kt0);
    issue(B1, kt0);
    issue(A1, kt0);
    issue(B0, kt0);
  }
  if (kt0 + 1 < kt1) {
    issue(A0, kt0 + 1);
    issue(B1, kt0 + 1);
    issue(A1, kt0 + 1);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");  // tile kt0 landed
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  bar();

  bf16x8 ra[2][4], rb0[2][2], rb1[2][2];
  auto read_a = [&](int buf, int h) {
    const char* img = himg(buf, h);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i) ra[kk][i] = frag<AKO>(img, wr * 64 + i * 16, kk);
  };
  auto read_b = [&](int buf, int h, bf16x8 (&rb)[2][2]) {
    const char* img = himg(buf, h);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int j = 0; j < 2; ++j) rb[kk][j] = frag<BKO>(img, wc * 32 + j * 16, kk);
  };
  // close a phase's load section: own ds_reads retired, then the barrier (see header)
  auto ready = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    bar();
  };
  auto quad = [&](int qm, int qn, const bf16x8 (&rb)[2][2]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[qm * 4 + i][qn * 2 + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(rb[kk][j], ra[kk][i], acc[qm * 4 + i][qn * 2 + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  if (wr == 1) bar();  // group 1 runs one barrier behind group 0
#pragma unroll 1
  for (int u = kt0; u < kt1; ++u) {
    const int buf = u & 1;
    // phase 0: Q(0,0) -- A0, B0 of tile u; restage B0(u+1)
    read_a(buf, A0);
    read_b(buf, B0, rb0);
    if (u + 1 < kt1) issue(B0, u + 1);
    ready();
    quad(0, 0, rb0);
    bar();
    // phase 1: Q(0,1) -- B1; restage A0(u+2)
    read_b(buf, B1, rb1);
    if (u + 2 < kt1) issue(A0, u + 2);
    ready();
    quad(0, 1, rb1);
    bar();
    // phase 2: Q(1,1) -- A1; restage B1(u+2)
    read_a(buf, A1);
    if (u + 2 < kt1) issue(B1, u + 2);
    ready();
    quad(1, 1, rb1);
    bar();
    // phase 3: Q(1,0) -- B0 again; restage A1(u+2); tile u+1 must be complete after this phase
    read_b(buf, B0, rb0);
    if (u + 2 < kt1) {
      issue(A1, u + 2);
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    ready();
    quad(1, 0, rb0);
    bar();
  }
  if (wr == 0) bar();  // re-align the groups: every wave has passed the same barrier count
  __syncthreads();
  constexpr int WPS = 2;  // waves per SIMD
  gemm_epilogue<BM, BN, NT, 2, EPI, (512 / WPS >= 256 ? 4 : 2), false, true>(p, acc, smem, m0, n0, bz);
}

}  // namespace g8

static int g_g8 = -1;
extern "C" void tfk_g8_set(int on) { g_g8 = on; }
static bool g8_on() {
  if (g_g8 < 0) g_g8 = 0;  // off until measured faster (tools/tile_ab.py)
  return g_g8 > 0;
}

// 256x256 GEMMs with K-inner A (fwd: B K-inner; dgrad: B K-outer) and the Cin % 64 == 0 conv
// forward gather (fwd, and stride-1 dgrad run as a forward conv with the BN-reduce epilogue).
// -1: not handled here.
extern "C" int tfk_g8_launch(const GemmParams& p_in, int amode, int bmode, int epi, int batch, int splits,
                             hipStream_t stream) {
  if (!g8_on()) return -1;
  const bool dense = (amode == g4::KIN && (bmode == g4::KIN || bmode == g4::KOUT)) ||
                     (amode == g4::KOUT && bmode == g4::KOUT && epi == EPI_F32);
  const bool conv = amode == g4::CONV_FWD && bmode == g4::KIN && (p_in.Cin & 63) == 0;
  if (!dense && !conv) return -1;
  GemmParams p = p_in;
  p.tiles_n = (p.N + g8::BN - 1) / g8::BN;
  const int tiles = ((p.M + g8::BM - 1) / g8::BM) * p.tiles_n;
  const dim3 grid(tiles, batch, splits), block(g8::NT);
#define TFK_G8(AM_, BMD_, EPI_)                                                                    \
  if (amode == AM_ && bmode == BMD_ && epi == EPI_) {                                              \
    hipLaunchKernelGGL((g8::g8_kernel<AM_, BMD_, EPI_>), grid, block, 0, stream, p);               \
    return hipGetLastError() == hipSuccess ? 0 : -2;                                               \
  }
  TFK_G8(g4::KIN, g4::KIN, EPI_BF16)
  TFK_G8(g4::KIN, g4::KIN, EPI_BF16_EXT)
  TFK_G8(g4::KIN, g4::KIN, EPI_F32)
  TFK_G8(g4::KIN, g4::KOUT, EPI_BF16)
  TFK_G8(g4::KIN, g4::KOUT, EPI_BF16_EXT)
  TFK_G8(g4::KIN, g4::KOUT, EPI_BF16_BNR)
  TFK_G8(g4::KOUT, g4::KOUT, EPI_F32)  // weight gradients dY^T X (split-K slabs by blockIdx.z)
  TFK_G8(g4::CONV_FWD, g4::KIN, EPI_BF16)
  TFK_G8(g4::CONV_FWD, g4::KIN, EPI_BF16_BNR)
#undef TFK_G8
  return -1;
}

}  // namespace tfk
