// Halo-tile direct 3x3 convolution for gfx950 (ResNet stage-1/2 3x3 convs: forward, and the
// stride-1 dgrad run as a forward conv over dY with flipped weights).
//
// The implicit-GEMM gather of the g4 engine (gemm_g4.hip A_CONV_FWD) DMAs one (tap, 64-channel)
// K-tile of gathered rows per step, so every input pixel is pulled from L2 nine times, and with a
// 64-wide B tile the 3x3 weights are re-read per 64 rows: measured 1.4 TB/s algorithmic, 12.9 TB/s
// of L2->LDS traffic at 56x56x64 (profiles/opprof_resnet50_bs256_r3a.txt: 0.145 ms fwd,
// 0.214 ms dgrad per layer). Here a block owns TR whole image rows x all W columns (GEMM rows =
// contiguous NHWC output pixels, so the shared g4 epilogue -- BN statistics / BN-backward reduce
// -- applies unchanged) and stages the (TR+2) x (W+2) halo of 64 input channels in LDS ONCE per
// channel chunk; the nine taps read their A fragments from the halo at shifted pixel offsets.
// Weights stream per (tap, chunk) K-tile through two LDS stages (g4 KIN loader).
//
// Halo image: pixel p (row-major over (TR+2) x (W+2)) is 128 B = 64 channels; 16-B chunk c of
// pixel p sits at p*128 + ((c ^ ((p >> 1) & 7)) << 4) -- the g4 K-inner swizzle, so the 16 lanes
// of a fragment read (16 consecutive pixels) are conflict-free except at the row wrap. Filled by
// LDS-DMA, 8 pixels (1 KiB) per wave instruction, swizzle applied to the per-lane SOURCE address;
// pixels outside the image read zeros (buffer range check) = the conv's zero padding.
#include "common.h"
#include "gemm_params.h"
#include "gemm_epilogue.h"
#include "g4_loader.h"

namespace tfk {
namespace halo {

using g4::BK;
using g4::NREC;
using g4::OOB;

template <int W, int TR>
struct Geo {
  static constexpr int BM = TR * W;               // GEMM rows per block (TR output image rows)
  static constexpr int HW2 = W + 2;               // halo row length (pad 1 each side)
  static constexpr int HPIX = (TR + 2) * HW2;     // halo pixels
  static constexpr int NDMA = (HPIX + 7) / 8;     // 1-KiB DMA instructions per halo fill
  static constexpr int HBYTES = NDMA * 1024;
};

__device__ __forceinline__ int hswz(int p) { return (p >> 1) & 7; }

// Fill one 64-channel halo image (chunk ch) of image n, output rows h0..h0+TR-1.
template <int W, int TR>
__device__ __forceinline__ void halo_issue(const GemmParams& p, char* img, int n, int h0, int ch, int w, int lane) {
  using G = Geo<W, TR>;
  __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)p.A, (short)0, NREC, 0x00020000);
  const int slot = lane & 7;
#pragma unroll
  for (int i = 0; i < (G::NDMA + 3) / 4; ++i) {
    const int j = 4 * i + w;  // wave-uniform
    if (j < G::NDMA) {
      const int pix = 8 * j + (lane >> 3);
      const int c = slot ^ hswz(pix);
      const int hr = pix / G::HW2, hc = pix - hr * G::HW2;
      const int h = h0 - 1 + hr, x = hc - 1;
      const bool ok = pix < G::HPIX && (unsigned)h < (unsigned)p.H && (unsigned)x < (unsigned)W;
      const unsigned vo =
          ok ? (unsigned)(((((long long)n * p.H + h) * W + x) * p.Cin + ch * 64 + c * 8) * 2) : OOB;
      lds_dma<16>(rsrc, (LDS_AS void*)(img + j * 1024), vo);
    }
  }
}

// A fragment (16 GEMM rows from the lane's base pixel, K-half kk) of tap offset `toff` (pixels).
__device__ __forceinline__ bf16x8 hfrag(const char* img, int pix0, int toff, int kk) {
  const int l = threadIdx.x & 63;
  const int pix = pix0 + toff;
  const int c = kk * 4 + (l >> 4);
  return *(const bf16x8*)(img + pix * 128 + ((c ^ hswz(pix)) << 4));
}

// W x TR rows per block, BN output channels, waves WM (rows) x WN (columns), 4 waves; CIN input
// channels (CH = CIN/64 halo chunks; 2 chunks: the next chunk's halo streams into a second image
// during the current chunk's 9 taps).
//
// Weights do NOT go through LDS: every wave loads its own B fragments (16 B per lane per fragment,
// L2-resident) straight into a D-deep register ring, D steps ahead of their MFMAs. With the halo
// resident the tap loop then has no barrier and no LDS-DMA wait at all (one per channel chunk for
// CIN = 128) -- the first version streamed each (tap, chunk) weight tile through LDS with a drain +
// barrier per tap and spent ~8x the MFMA time of a tap waiting on L2 latency.
template <int W, int TR, int CIN, int BN, int WM, int WN, int EPI>
__global__ __launch_bounds__(256, 2) void hconv_kernel(GemmParams p) {
  using G = Geo<W, TR>;
  constexpr int NW = 4, NTH = 256, BM = G::BM;
  static_assert(WM * WN == NW, "4 waves");
  constexpr int TM = BM / WM, TN = BN / WN, FM = TM / 16, FN = TN / 16;
  static_assert(TM % 16 == 0 && TN % 16 == 0, "fragment tiling");
  constexpr int CH = CIN / 64, NSTEP = 9 * CH, HB = CH > 1 ? 2 : 1;
  constexpr int D = 3;  // B-fragment prefetch depth (steps)
  constexpr int MAIN = HB * G::HBYTES, EPIB = epi_lds_bytes<BM, BN, WM>();
  __shared__ __attribute__((aligned(16))) char smem[MAIN > EPIB ? MAIN : EPIB];

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w / WN, wn = w % WN;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);  // neighbouring row bands share an XCD's L2
  const int mt = tile / p.tiles_n, nt = tile - mt * p.tiles_n;
  const int m0 = mt * BM, n0 = nt * BN;
  const int HWp = p.H * W;
  const int n = m0 / HWp, h0 = (m0 - n * HWp) / W;
  auto himg = [&](int i) { return smem + (i & (HB - 1)) * G::HBYTES; };

  // halo pixel of tap (0,0) for each A fragment's row of this lane
  int pix0[FM];
#pragma unroll
  for (int f = 0; f < FM; ++f) {
    const int r = wm * TM + f * 16 + (lane & 15);
    const int rr = r / W, cc = r - rr * W;
    pix0[f] = rr * G::HW2 + cc;
  }
  // this lane's B fragment rows: W[n0 + wn*TN + j*16 + (lane&15)][k], k = tap*CIN + ch*64 + chunk*8
  const bf16* brow = (const bf16*)p.B + (long long)(n0 + wn * TN + (lane & 15)) * p.ldb + (lane >> 4) * 8;
  bf16x8 breg[D][2][FN];
  auto bload = [&](int s, bf16x8 (&dst)[2][FN]) {
    const int ch = s / 9, tap = s - ch * 9;
    const bf16* b = brow + tap * CIN + ch * 64;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int j = 0; j < FN; ++j) dst[kk][j] = *(const bf16x8*)(b + (long long)j * 16 * p.ldb + kk * 32);
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  halo_issue<W, TR>(p, himg(0), n, h0, 0, w, lane);
#pragma unroll
  for (int s = 0; s < D; ++s) bload(s, breg[s]);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

#pragma unroll
  for (int s = 0; s < NSTEP; ++s) {
    const int ch = s / 9, tap = s - ch * 9;
    if (s > 0 && tap == 0) {
      // chunk boundary (CIN = 128): the halo issued 9 taps ago has landed for every wave
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
    if (HB == 2 && tap == 0 && ch + 1 < CH) halo_issue<W, TR>(p, himg(ch + 1), n, h0, ch + 1, w, lane);
    const char* hs = himg(ch);
    const int toff = (tap / 3) * G::HW2 + (tap % 3);
    // all of the tap's A fragments are read before its MFMAs: issued back to back, the ds_reads
    // overlap each other and the first MFMAs wait for one fragment only (read-then-use per
    // fragment exposed the LDS latency on every pair of MFMAs)
    bf16x8 a[2][FM];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int f = 0; f < FM; ++f) a[kk][f] = hfrag(hs, pix0[f], toff, kk);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
      for (int f = 0; f < FM; ++f) {
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[f][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(breg[s % D][kk][j], a[kk][f], acc[f][j], 0, 0, 0);
      }
    }
    if (s + D < NSTEP) bload(s + D, breg[s % D]);
  }
  __syncthreads();
  gemm_epilogue<BM, BN, NTH, WM, EPI, 2>(p, acc, smem, m0, n0, 0);
}

}  // namespace halo

static int g_halo = -1;
static bool halo_on() {
  if (g_halo < 0) {
    const char* e = getenv("TFK_HALO");
    g_halo = e ? atoi(e) : 1;  // 0 off, 1 stage-1 shapes, 2 + stage-2 shapes
  }
  return g_halo >= 1;
}

// Launch the halo kernel when the conv is a 3x3 / stride 1 / pad 1 / undilated forward conv of a
// supported (W, Cout) shape with a bf16 (stats) or BN-backward-reduce epilogue; -1 otherwise.
extern "C" int tfk_halo_launch(const GemmParams& p_in, int epi, int batch, int splits, hipStream_t stream) {
  if (!halo_on() || batch != 1 || splits != 1) return -1;
  const GemmParams& q = p_in;
  if (q.R != 3 || q.S != 3 || q.sh != 1 || q.sw != 1 || q.ph != 1 || q.pw != 1 || q.dh != 1 || q.dw != 1) return -1;
  if (q.P != q.H || q.Q != q.W || (q.Cin & 63) || q.om_hp != 0 || q.rs_sh != 0) return -1;
  if (epi != EPI_BF16 && epi != EPI_BF16_BNR) return -1;
  if (q.ldb != 9LL * q.Cin || q.ldc != q.N || q.K != 9 * q.Cin || ((uintptr_t)q.A & 15) || ((uintptr_t)q.B & 15)) return -1;
  if ((long long)q.Nimg * q.H * q.W * q.Cin >= (1LL << 30)) return -1;
  GemmParams p = p_in;
#define TFK_HALO_CASE(W_, TR_, CIN_, BN_, WM_, WN_)                                                     \
  if (q.W == W_ && q.Cin == CIN_ && q.H % TR_ == 0 && q.N % BN_ == 0) {                                \
    p.tiles_n = q.N / BN_;                                                                              \
    const int tiles = (q.Nimg * q.H / TR_) * p.tiles_n;                                                 \
    if (epi == EPI_BF16)                                                                                \
      hipLaunchKernelGGL((halo::hconv_kernel<W_, TR_, CIN_, BN_, WM_, WN_, EPI_BF16>), dim3(tiles), dim3(256), 0,  \
                         stream, p);                                                                    \
    else                                                                                                \
      hipLaunchKernelGGL((halo::hconv_kernel<W_, TR_, CIN_, BN_, WM_, WN_, EPI_BF16_BNR>), dim3(tiles), dim3(256),  \
                         0, stream, p);                                                                 \
    return hipGetLastError() == hipSuccess ? 0 : -2;                                                    \
  }
  // ResNet stage 1 (56x56, 64 -> 64): 4 image rows = 224 GEMM rows x 64 channels, 2 x 2 waves,
  // one 44-KiB halo image
  if (q.N == 64) TFK_HALO_CASE(56, 4, 64, 64, 2, 2)
  // ResNet stage 2 (28x28, 128 -> 128; 4 rows = 112 rows x 128 channels, 1 x 4 waves, two 23-KiB
  // halo images) measured level with the gather (fwd 0.101 vs 0.101 ms, dgrad 0.133 vs 0.135 ms,
  // tools/halo_bench.py): 228 VGPRs leave 2 waves/SIMD. Opt-in TFK_HALO=2 until it wins.
  if (q.N == 128 && g_halo == 2) TFK_HALO_CASE(28, 4, 128, 128, 1, 4)
#undef TFK_HALO_CASE
  return -1;
}
extern "C" void tfk_halo_set(int on) { g_halo = on < 0 ? -1 : on; }

}  // namespace tfk
