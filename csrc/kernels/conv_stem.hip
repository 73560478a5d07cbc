// ResNet stem forward for gfx950: 7x7 / stride 2 / pad 3 conv of an RGB image padded to 8
// channels (x [N][224][224][8], channels >= 4 zero) into 64 channels, with the BN batch statistics
// in the epilogue (gemm_epilogue.h EPI_BF16 + stats).
//
// The implicit-GEMM gather on the g4 engine (Loader CONV_FWD, Cin < 64) runs K = 49 taps x 8
// channels of which 5/8 are zero padding, DMAs an im2col tile per K-step (every input pixel ~12x
// through L2 -> LDS) and reached 24% of roofline (0.43 ms of a 23 ms step,
// profiles/opprof_resnet50_bs256_r3a.txt). Here a block owns a band of TR = 2 output rows (224
// GEMM rows = 224 pixels), stages the 9 x 229 input halo ONCE by LDS-DMA (16-B pixels; even and
// odd columns split so the 16 output pixels of a fragment read 16 consecutive halo pixels), and
// runs K = 56 taps x 4 channels (49 real taps, 3 real channels + 1 zero): each lane's 8 k-elements
// of a step are channels 0..3 of two taps = two 8-byte LDS reads at per-lane tap offsets. Weights
// live in registers (each wave's 32 output channels x 7 k-steps, loaded once from L2). The output
// write (411 MB at bs256) is the floor.
#include "common.h"
#include "gemm_params.h"
#include "gemm_epilogue.h"
#include "g4_loader.h"

namespace tfk {
namespace stemf {

using g4::NREC;
using g4::OOB;

template <int Q, int TR>
struct Geo {
  static constexpr int HR = (TR - 1) * 2 + 7;
  static constexpr int HCR = (Q - 1) * 2 + 7;
  static constexpr int HALF = ((Q + 3) + 15) / 16 * 16 + 4;
  static constexpr int HC = 2 * HALF;
  static constexpr int XPIX = (HR * HC + 63) / 64 * 64;
  static constexpr int BM = TR * Q;
  static constexpr int NKS = 7;  // 56 taps x 4 channels / 32
};

// 4 waves: 2 (output rows of the band) x 2 (32-channel halves); wave tile Q x 32.
template <int Q, int TR>
__global__ __launch_bounds__(256, 2) void stem_fwd_kernel(GemmParams p, int bands_per_img) {
  using G = Geo<Q, TR>;
  static_assert(TR == 2, "wave rows = band rows");
  constexpr int BM = G::BM, BN = 64, WM = 2, FM = Q / 16, FN = 2;
  constexpr int EPIB = epi_lds_bytes<BM, BN, WM>(), XB = G::XPIX * 16;
  __shared__ __attribute__((aligned(16))) char smem[XB > EPIB ? XB : EPIB];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 1, wn = w & 1;
  const int g = lane >> 4;
  // neighbouring bands (7 of their 9 halo rows shared) on one XCD: the shared rows hit its L2
  const int bd = xcd_remap(blockIdx.x, gridDim.x);
  const int n = bd / bands_per_img, h0 = (bd - n * bands_per_img) * TR;

  // halo DMA: 64 pixels (1 KiB) per wave instruction, zero outside the image (= the conv padding)
  {
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)p.A, (short)0, NREC, 0x00020000);
#pragma unroll
    for (int it = 0; it < (G::XPIX / 64 + 3) / 4; ++it) {
      const int jd = 4 * it + w;
      if (jd < G::XPIX / 64) {
        const int pix = 64 * jd + lane;
        const int hr = pix / G::HC, hp = pix - hr * G::HC;
        const int ph = hp >= G::HALF, hc = 2 * (hp - ph * G::HALF) + ph;
        const int hh = 2 * h0 - 3 + hr, ww = hc - 3;
        const bool ok = hr < G::HR && hc < G::HCR && (unsigned)hh < (unsigned)p.H && (unsigned)ww < (unsigned)p.W;
        const unsigned vo = ok ? (unsigned)((((long long)n * p.H + hh) * p.W + ww) * 16) : OOB;
        lds_dma<16>(rx, (LDS_AS void*)(smem + jd * 1024), vo);
      }
    }
  }

  // weights: lane (co = 32wn + 16j + (l&15), k-group g) of step ks holds channels 0..3 of taps
  // 8ks + 2g and 8ks + 2g + 1 (taps >= 49: zero); w is [64][49][8] bf16
  bf16x8 bw[G::NKS][FN];
  const bf16* wb = (const bf16*)p.B;
#pragma unroll
  for (int ks = 0; ks < G::NKS; ++ks)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int co = 32 * wn + 16 * j + (lane & 15);
      const int t0 = 8 * ks + 2 * g;
      bf16x4 lo = {}, hi = {};
      if (t0 < 49) lo = *(const bf16x4*)(wb + (co * 49 + t0) * 8);
      if (t0 + 1 < 49) hi = *(const bf16x4*)(wb + (co * 49 + t0 + 1) * 8);
      bw[ks][j].lo = lo;
      bw[ks][j].hi = hi;
    }
  // per-lane halo byte offsets of the two taps of each k-step (taps >= 49 clamped: zero weights)
  int to[G::NKS][2];
#pragma unroll
  for (int ks = 0; ks < G::NKS; ++ks)
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      int t = 8 * ks + 2 * g + e;
      t = t < 49 ? t : 48;
      const int r = t / 7, s = t - r * 7;
      to[ks][e] = (r * G::HC + (s & 1) * G::HALF + (s >> 1)) * 16;
    }
  const int base = (2 * wm * G::HC + (lane & 15)) * 16;  // output row wm of the band, column l&15

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

#pragma unroll
  for (int ks = 0; ks < G::NKS; ++ks) {
    bf16x8 a[FM];
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const char* pa = smem + base + i * 16 * 16;  // 16 output columns = 16 halo pixels per fragment
      a[i].lo = *(const bf16x4*)(pa + to[ks][0]);
      a[i].hi = *(const bf16x4*)(pa + to[ks][1]);
    }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[ks][j], a[i], acc[i][j], 0, 0, 0);
  }
  __syncthreads();  // every wave is done with the halo: the epilogue reuses the LDS
  gemm_epilogue<BM, BN, 256, WM, EPI_BF16, 2>(p, acc, smem, bd * BM, 0, 0);
}

}  // namespace stemf
}  // namespace tfk

using namespace tfk;

// y [N][H/2][W/2][64] = conv7x7/s2/p3(x [N][H][W][8], w [64][7][7][8]) (channels >= 4 of x zero),
// stats [shards][2][64] += per-channel (sum, sumsq). W must be 224 (Q = 112), H % 4 == 0.
extern "C" int tfk_stem_fwd_ok(int N, int H, int W) {
  return W == 224 && H % 4 == 0 && N >= 1 && (long long)N * H * W * 16 < 0x7FFFFFF0LL;
}
extern "C" int tfk_stem_fwd_launch(const void* x, const void* w, void* y, float* stats, int shards, int N, int H, int W,
                                   hipStream_t stream) {
  if (!tfk_stem_fwd_ok(N, H, W)) return -1;
  GemmParams p{};
  p.A = x;
  p.B = w;
  p.C = y;
  p.P = H / 2;
  p.Q = W / 2;
  p.M = N * p.P * p.Q;
  p.N = 64;
  p.K = 49 * 8;
  p.ldc = 64;
  p.alpha = 1.f;
  p.beta = 0.f;
  p.stats = stats;
  p.stats_shards = shards < 1 ? 1 : shards;
  p.Nimg = N;
  p.H = H;
  p.W = W;
  p.Cin = 8;
  p.Cout = 64;
  const int bpi = p.P / 2;
  hipLaunchKernelGGL((stemf::stem_fwd_kernel<112, 2>), dim3(N * bpi), dim3(256), 0, stream, p, bpi);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
