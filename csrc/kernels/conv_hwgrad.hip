// Halo-tile direct weight gradient of 3x3 convolutions (pad 1, stride 1 or 2) for gfx950: every
// 3x3 conv of ResNet-50/101/152.
//
//   dW[co][r][s][ci] = sum over output pixels (n, i, j) of dY[n,i,j,co] * X[n, i*st-1+r, j*st-1+s, ci]
//
// The implicit-GEMM path (g4 engine, B_CONV_WGRAD) DMAs an im2col K-tile of gathered pixels per
// (tap, channel) column block, so every input pixel crosses L2->LDS nine times and dY once per
// 128-column block: 19-27% of the MFMA roofline on every 3x3 weight gradient of ResNet-50
// (profiles/opprof_resnet50_bs256_r3a.txt: 0.205 ms per 56x56x64 layer, 2.0 ms per step in all).
//
// Here a block owns one (64 output-channel, 64 input-channel) chunk pair and ALL nine taps (a
// 64 x 576 slice of dW, 18 f32x4 accumulators per wave) and walks "bands" of output pixels: TR
// whole output rows of NB images. Per band the (TR-1)*st+3 input rows x all columns of 64 input
// channels (the halo) and the band's dY rows of 64 output channels are DMA'd into LDS once (two
// stages: band t+1 lands while band t computes); the GEMM's K = band pixels, 32 per MFMA step.
// Both operands are read with ds_read_b64_tr_b16 (cdna_hip_programming.md T10): each lane supplies
// the address of ITS k-row, so the im2col shift of a tap is just a different per-lane pixel
// offset into the halo -- no gather, no re-load per tap. Partial sums of a block go to its own f32
// slab; splitk_reduce folds the slabs into the gradient (bitwise deterministic).
//
// LDS images: pixel rows of 128 B (64 channels). Tr reads of one 32-lane half touch 8 pixel rows
// (k rows k0..k0+3, k0+8..k0+11) x 32 B, so the swizzle permutes the four 32-B channel PAIRS of a
// row by f(P>>1) = bit0 | bit2<<1: rows P, P+2, P+8, P+10 (same bank parity) get four distinct
// pairs for ANY start offset -> conflict-free. Stride 2 stores even input columns before odd ones
// (phase split), so the pixels of a tap's 8 rows are consecutive again. Halo rows are padded to a
// multiple of 16 pixels: a tap-row shift r*HC then leaves the swizzle bits unchanged, and the
// per-lane offsets of the three column taps are precomputed once per kernel.
#include "common.h"
#include "g4_loader.h"

namespace tfk {
namespace hwg {

using g4::NREC;
using g4::OOB;

struct HWParams {
  const bf16* x;   // [Nimg][H][W][C]
  const bf16* dy;  // [Nimg][P][Q][K]
  float* ws;       // [slabs][K][3][3][C]
  int Nimg, H, W, P, C, K;
  int nbands, bands_per_img, bands_per_block;
  long long slab;  // floats per slab
};

__device__ __forceinline__ int pswz(int P) {
  const int a = P >> 1;
  return (a & 1) | (((a >> 2) & 1) << 1);
}

template <int Q, int TR, int NB, int ST>
struct Geo {
  static constexpr int HR = (TR - 1) * ST + 3;          // halo rows per image
  static constexpr int HCR = (Q - 1) * ST + 3;          // real halo columns
  static constexpr int HALF = ((Q + 1) + 7) / 8 * 8;  // stride 2: even / odd column halves
  static constexpr int HC = ST == 1 ? (HCR + 15) / 16 * 16 : 2 * HALF;
  static constexpr int XPIX = NB * HR * HC;
  static constexpr int NPIX = NB * TR * Q;               // band output pixels = GEMM K per band
  static constexpr int NKS = (NPIX + 31) / 32;           // MFMA k-steps per band
  static constexpr int DROWS = (NPIX + 1 + 7) / 8 * 8;   // + zero row NPIX (padded k)
  static constexpr int XB = XPIX * 128, DB = DROWS * 128, STAGE = XB + DB;
  static_assert(2 * STAGE <= 160 * 1024, "two stages must fit the 160 KiB LDS");
  static_assert(XPIX % 8 == 0, "DMA granularity");
};

template <int Q, int TR, int NB, int ST>
__global__ __launch_bounds__(512, 1) void hwgrad_kernel(HWParams p) {
  using G = Geo<Q, TR, NB, ST>;
  __shared__ __attribute__((aligned(16))) char smem[2 * G::STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = w >> 2, wn = w & 3;  // wave: output-channel half (2 x 16), input-channel group of 16
  // block -> (band range bx, chunk pair y): XCD-contiguous logical ids, pairs fastest, so the
  // blocks sharing a band range (same halo / dY rows, other channel chunks) share one XCD's L2
  const int npairs = (p.K >> 6) * (p.C >> 6);
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int bx = lid / npairs, by = lid - bx * npairs;
  const int nci = p.C >> 6;
  const int co0 = (by / nci) * 64, ci0 = (by % nci) * 64;
  const int g = lane >> 4, q = (lane >> 2) & 3, pl = lane & 3;

  // per-lane LDS byte offsets of this lane's tr-read row: X for column taps s = 0..2 (row taps add
  // r*HC pixels), dY for the wave's first output-channel fragment (the second one: ^ 32)
  int xo[3][G::NKS][2], dofs[G::NKS][2];
#pragma unroll
  for (int ks = 0; ks < G::NKS; ++ks)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = ks * 32 + 8 * g + 4 * h + q;
      int b = 0, i = 0, j = 0, drow = G::NPIX;
      if (k < G::NPIX) {
        b = k / (TR * Q);
        const int rem = k - b * TR * Q;
        i = rem / Q;
        j = rem - i * Q;
        drow = k;
      }
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        int P;
        if constexpr (ST == 1) P = b * G::HR * G::HC + i * G::HC + j + s;
        else P = b * G::HR * G::HC + (2 * i) * G::HC + (s & 1) * G::HALF + j + (s >> 1);
        xo[s][ks][h] = P * 128 + ((wn ^ pswz(P)) << 5) + pl * 8;
      }
      dofs[ks][h] = G::XB + drow * 128 + (((2 * wc) ^ pswz(drow)) << 5) + pl * 8;
    }

  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, NREC, 0x00020000);
  const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc((void*)p.dy, (short)0, NREC, 0x00020000);
  const int slot = lane & 7;
  auto issue = [&](int bd, char* img) {
    int n0, h0;
    if constexpr (NB == 1) {
      n0 = bd / p.bands_per_img;
      h0 = (bd - n0 * p.bands_per_img) * TR;
    } else {
      n0 = bd * NB;
      h0 = 0;
    }
#pragma unroll
    for (int it = 0; it < (G::XPIX / 8 + 7) / 8; ++it) {
      const int jd = 8 * it + w;  // wave-uniform
      if (jd < G::XPIX / 8) {
        const int pix = 8 * jd + (lane >> 3);
        const int c = slot ^ (pswz(pix) << 1);
        const int b = pix / (G::HR * G::HC), rem = pix - b * G::HR * G::HC;
        const int hr = rem / G::HC, hp = rem - hr * G::HC;
        const int col = ST == 1 ? hp : (hp < G::HALF ? 2 * hp : 2 * (hp - G::HALF) + 1);
        const int n = n0 + b, hh = h0 * ST - 1 + hr, ww = col - 1;
        const bool ok = n < p.Nimg && col < G::HCR && (unsigned)hh < (unsigned)p.H && (unsigned)ww < (unsigned)p.W;
        const unsigned vo = ok ? (unsigned)(((((long long)n * p.H + hh) * p.W + ww) * p.C + ci0 + c * 8) * 2) : OOB;
        lds_dma<16>(rx, (LDS_AS void*)(img + jd * 1024), vo);
      }
    }
    const long long pix0 = ((long long)n0 * p.P + h0) * Q;
    const long long npx = (long long)p.Nimg * p.P * Q;
#pragma unroll
    for (int it = 0; it < (G::DROWS / 8 + 7) / 8; ++it) {
      const int jd = 8 * it + w;
      if (jd < G::DROWS / 8) {
        const int r = 8 * jd + (lane >> 3);
        const int c = slot ^ (pswz(r) << 1);
        const bool ok = r < G::NPIX && pix0 + r < npx;
        const unsigned vo = ok ? (unsigned)(((pix0 + r) * p.K + co0 + c * 8) * 2) : OOB;
        lds_dma<16>(rd, (LDS_AS void*)(img + G::XB + jd * 1024), vo);
      }
    }
  };

  f32x4 acc[9][2];
#pragma unroll
  for (int t = 0; t < 9; ++t) acc[t][0] = acc[t][1] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto tr = [](const char* a) { return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((LDS_AS bf16x4*)a); };
  auto compute = [&](const char* img) {
#pragma unroll
    for (int ks = 0; ks < G::NKS; ++ks) {
      bf16x8 a0, a1;
      a0.lo = tr(img + dofs[ks][0]);
      a0.hi = tr(img + dofs[ks][1]);
      a1.lo = tr(img + (dofs[ks][0] ^ 32));
      a1.hi = tr(img + (dofs[ks][1] ^ 32));
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int r = tap / 3, s = tap % 3;
        bf16x8 bx;
        bx.lo = tr(img + xo[s][ks][0] + r * G::HC * 128);
        bx.hi = tr(img + xo[s][ks][1] + r * G::HC * 128);
        acc[tap][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bx, a0, acc[tap][0], 0, 0, 0);
        acc[tap][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bx, a1, acc[tap][1], 0, 0, 0);
      }
    }
  };

  // a contiguous range of bands per block: the halo rows two neighbouring bands share come from L2
  const int b0 = bx * p.bands_per_block, b1 = min(p.nbands, b0 + p.bands_per_block);
  if (b0 < b1) issue(b0, smem);
#pragma unroll 1
  for (int bd = b0; bd < b1; ++bd) {
    const int t = bd - b0;
    char* cur = smem + (t & 1) * G::STAGE;
    // band t landed; every wave finished band t-1, whose stage the next DMA overwrites
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (bd + 1 < b1) issue(bd + 1, smem + ((t + 1) & 1) * G::STAGE);
    compute(cur);
  }

  // slab store: lane holds D[ci 4*(l>>4)+0..3][co l&15] of fragment (tap, co half t)
  float* out = p.ws + (long long)bx * p.slab;
  const int C9 = 9 * p.C;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int co = co0 + 32 * wc + 16 * t + (lane & 15);
#pragma unroll
    for (int tap = 0; tap < 9; ++tap)
      *(f32x4*)(out + (long long)co * C9 + tap * p.C + ci0 + 16 * wn + 4 * (lane >> 4)) = acc[tap][t];
  }
}

}  // namespace hwg

// ---------------------------------------------------------------------------------------------
// Stem weight gradient: 7x7 / stride 2 / pad 3 conv of an 8-channel-padded RGB image (ResNet
// conv1: x [N][224][224][8], channels >= 4 zero; dy [N][112][112][64]). The im2col gather on the
// g4 engine computes all 8 padded channels (N = 49 x 8 = 392 columns, 5/8 of them zero) at 17% of
// roofline (0.64 ms/step, the last kernel of the backward). Here the GEMM's columns are (tap,
// channel 0..3): ONE 8-byte tr16 read per lane and k-row = 4 channels of a tap, so a 16-column
// fragment is 4 taps (13 fragments for 49 taps instead of 25) and the zero channels 4..7 are only
// stored. Bands are TR = 2 output rows (224 pixels = 7 MFMA k-steps) of one image; the 9 input rows
// x 229 columns halo (16-B pixels, even/odd columns split so a tap's 16 consecutive output pixels
// read 16 consecutive halo pixels) and the band's dY rows land by LDS-DMA in two stages. Each block
// walks one contiguous run of bands (one image at bs256 on 256 CUs), so the 7 halo rows two bands
// share come from L2 and HBM sees x and dY about once: dY's 411 MB at bs256 is the floor.
// 8 waves: 2 (output-channel halves) x 4 (column groups of 4 fragments = 16 taps; taps >= 49 are
// computed on clamped addresses and dropped).
namespace stem {

using g4::NREC;
using g4::OOB;

template <int Q, int TR>
struct Geo {
  static constexpr int HR = (TR - 1) * 2 + 7;
  static constexpr int HCR = (Q - 1) * 2 + 7;                  // real halo columns (pad 3 + 3)
  static constexpr int HALF = ((Q + 3) + 15) / 16 * 16 + 4;   // even / odd halves; 16*HALF = 64 mod 256
  static constexpr int HC = 2 * HALF;
  static constexpr int XPIX = (HR * HC + 63) / 64 * 64;       // 64 pixels (1 KiB) per DMA instruction
  static constexpr int NPIX = TR * Q;
  static constexpr int NKS = (NPIX + 31) / 32;
  static constexpr int DROWS = (NPIX + 1 + 7) / 8 * 8;
  static constexpr int XB = XPIX * 16, DB = DROWS * 128, STAGE = XB + DB;
  static_assert(2 * STAGE <= 160 * 1024, "two stages must fit the 160 KiB LDS");
};

struct SParams {
  const bf16* x;   // [Nimg][H][W][8]
  const bf16* dy;  // [Nimg][P][Q][64]
  float* ws;       // [slabs][64][7][7][8]
  int Nimg, H, W, P;
  int nbands, bands_per_img, bands_per_block;
};

template <int Q, int TR>
__global__ __launch_bounds__(512, 1) void stem_wgrad_kernel(SParams p) {
  using G = Geo<Q, TR>;
  __shared__ __attribute__((aligned(16))) char smem[2 * G::STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = w >> 2, wn = w & 3;
  const int g = lane >> 4, q = (lane >> 2) & 3, pl = lane & 3;
  const int bx = xcd_remap(blockIdx.x, gridDim.x);

  // this lane's tap of each of the wave's 4 column fragments (fragment f = 4wn + ff: taps 4f..4f+3)
  int toff[4];
#pragma unroll
  for (int ff = 0; ff < 4; ++ff) {
    int t = 4 * (4 * wn + ff) + pl;
    t = t < 49 ? t : 48;
    const int r = t / 7, s = t - r * 7;
    toff[ff] = (r * G::HC + (s & 1) * G::HALF + (s >> 1)) * 16;
  }
  int xb[G::NKS][2], dofs[G::NKS][2];
#pragma unroll
  for (int ks = 0; ks < G::NKS; ++ks)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = ks * 32 + 8 * g + 4 * h + q;
      int pix = 0, drow = G::NPIX;
      if (k < G::NPIX) {
        const int i = k / Q, j = k - i * Q;
        pix = 2 * i * G::HC + j;
        drow = k;
      }
      xb[ks][h] = pix * 16;
      dofs[ks][h] = G::XB + drow * 128 + (((2 * wc) ^ hwg::pswz(drow)) << 5) + pl * 8;
    }

  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, NREC, 0x00020000);
  const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc((void*)p.dy, (short)0, NREC, 0x00020000);
  auto issue = [&](int bd, char* img) {
    const int n = bd / p.bands_per_img, h0 = (bd - n * p.bands_per_img) * TR;
#pragma unroll
    for (int it = 0; it < (G::XPIX / 64 + 7) / 8; ++it) {
      const int jd = 8 * it + w;  // wave-uniform
      if (jd < G::XPIX / 64) {
        const int pix = 64 * jd + lane;
        const int hr = pix / G::HC, hp = pix - hr * G::HC;
        const int ph = hp >= G::HALF, hc = 2 * (hp - ph * G::HALF) + ph;
        const int hh = 2 * h0 - 3 + hr, ww = hc - 3;
        const bool ok = hr < G::HR && hc < G::HCR && (unsigned)hh < (unsigned)p.H && (unsigned)ww < (unsigned)p.W;
        const unsigned vo = ok ? (unsigned)((((long long)n * p.H + hh) * p.W + ww) * 16) : OOB;
        lds_dma<16>(rx, (LDS_AS void*)(img + jd * 1024), vo);
      }
    }
    const long long pix0 = ((long long)n * p.P + h0) * Q;
    const int slot = lane & 7;
#pragma unroll
    for (int it = 0; it < (G::DROWS / 8 + 7) / 8; ++it) {
      const int jd = 8 * it + w;
      if (jd < G::DROWS / 8) {
        const int r = 8 * jd + (lane >> 3);
        const int c = slot ^ (hwg::pswz(r) << 1);
        const unsigned vo = r < G::NPIX ? (unsigned)(((pix0 + r) * 64 + c * 8) * 2) : OOB;
        lds_dma<16>(rd, (LDS_AS void*)(img + G::XB + jd * 1024), vo);
      }
    }
  };

  f32x4 acc[4][2];
#pragma unroll
  for (int f = 0; f < 4; ++f) acc[f][0] = acc[f][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto tr = [](const char* a) { return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((LDS_AS bf16x4*)a); };
  auto compute = [&](const char* img) {
#pragma unroll
    for (int ks = 0; ks < G::NKS; ++ks) {
      bf16x8 a0, a1;
      a0.lo = tr(img + dofs[ks][0]);
      a0.hi = tr(img + dofs[ks][1]);
      a1.lo = tr(img + (dofs[ks][0] ^ 32));
      a1.hi = tr(img + (dofs[ks][1] ^ 32));
#pragma unroll
      for (int ff = 0; ff < 4; ++ff) {
        bf16x8 bx;
        bx.lo = tr(img + xb[ks][0] + toff[ff]);
        bx.hi = tr(img + xb[ks][1] + toff[ff]);
        acc[ff][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bx, a0, acc[ff][0], 0, 0, 0);
        acc[ff][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bx, a1, acc[ff][1], 0, 0, 0);
      }
    }
  };

  const int b0 = bx * p.bands_per_block, b1 = min(p.nbands, b0 + p.bands_per_block);
  if (b0 < b1) issue(b0, smem);
#pragma unroll 1
  for (int bd = b0; bd < b1; ++bd) {
    const int t = bd - b0;
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (bd + 1 < b1) issue(bd + 1, smem + ((t + 1) & 1) * G::STAGE);
    compute(smem + (t & 1) * G::STAGE);
  }

  // lane holds D[(tap 4f + (l>>4)), channels 0..3][co l&15]; channels 4..7 (zero padding) get 0
  float* out = p.ws + (long long)bx * (64 * 49 * 8);
#pragma unroll
  for (int ff = 0; ff < 4; ++ff) {
    const int tap = 4 * (4 * wn + ff) + g;
    if (tap < 49) {
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        float* d = out + (32 * wc + 16 * t + (lane & 15)) * 392 + tap * 8;
        *(f32x4*)d = acc[ff][t];
        *(f32x4*)(d + 4) = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  }
}

}  // namespace stem

// (TR, NB) band shape served for an output width Q and stride st; false when none.
static bool hwg_shape(int Q, int P, int st, int* TR, int* NB) {
  struct S { int q, st, tr, nb; };
  static const S tab[] = {{56, 1, 4, 1}, {28, 1, 7, 1}, {14, 1, 14, 1}, {7, 1, 7, 3},
                          {28, 2, 2, 1}, {14, 2, 7, 1}};
  // (Q 7, stride 2: 7x7 from 14x14x512, 2-image bands) measured 0.110 vs 0.096 ms for the gather
  // (profiles/hwgrad_bench_r3.jsonl): not served
  for (const S& e : tab)
    if (e.q == Q && e.st == st && (e.nb == 1 ? P % e.tr == 0 : P == e.tr)) {
      *TR = e.tr;
      *NB = e.nb;
      return true;
    }
  return false;
}

// Bands of output pixels and slabs (blocks per chunk pair) of a conv; 0 slabs = not served.
// x [Nimg][H][W][C], dy [Nimg][P][Q][K], 3x3 / pad 1 / stride st.
static int hwg_plan(int H, int W, int P, int Q, int C, int K, int st, int Nimg, int* nbands, int* bpi) {
  int TR, NB;
  if ((C & 63) || (K & 63) || (st != 1 && st != 2) || Nimg < 1) return 0;
  if (P != (H - 1) / st + 1 || Q != (W - 1) / st + 1) return 0;
  if ((long long)Nimg * H * W * C * 2 >= 0x7FFFFFF0LL || (long long)Nimg * P * Q * K * 2 >= 0x7FFFFFF0LL) return 0;
  if (!hwg_shape(Q, P, st, &TR, &NB)) return 0;
  *bpi = NB == 1 ? P / TR : 1;
  *nbands = NB == 1 ? Nimg * (P / TR) : (Nimg + NB - 1) / NB;
  // ~one block per CU in all (256 CUs): chunk pairs x slabs
  const int npairs = (K / 64) * (C / 64);
  int gx = 256 / npairs;
  if (gx < 1) gx = 1;
  if (gx > *nbands) gx = *nbands;
  return gx;
}

}  // namespace tfk

using namespace tfk;

// Stem 7x7/s2/p3 weight gradient (x [N][H][W][8] with channels >= 4 zero, dy [N][H/2][W/2][64]):
// slabs = blocks (0: not served). One block per image when N >= 256.
static int stem_plan(int N, int H, int W, int* bpi, int* nbands, int* bpb) {
  if (W != 224 || H % 4 != 0 || N < 1 || (long long)N * H * W * 16 >= 0x7FFFFFF0LL) return 0;
  const int P = H / 2;
  *bpi = P / 2;
  *nbands = N * *bpi;
  int gx = N < 256 ? N : 256;
  *bpb = (*nbands + gx - 1) / gx;
  return gx;
}
extern "C" int tfk_stem_wgrad_slabs(int N, int H, int W) {
  int a, b, c;
  return stem_plan(N, H, W, &a, &b, &c);
}
extern "C" int tfk_stem_wgrad_launch(const void* x, const void* dy, float* ws, int N, int H, int W, int slabs,
                                     hipStream_t stream) {
  stem::SParams p;
  const int gx = stem_plan(N, H, W, &p.bands_per_img, &p.nbands, &p.bands_per_block);
  if (gx < 1 || gx != slabs) return -1;
  p.x = (const bf16*)x;
  p.dy = (const bf16*)dy;
  p.ws = ws;
  p.Nimg = N;
  p.H = H;
  p.W = W;
  p.P = H / 2;
  hipLaunchKernelGGL((stem::stem_wgrad_kernel<112, 2>), dim3(gx), dim3(512), 0, stream, p);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

extern "C" int tfk_hwgrad_slabs(int H, int W, int P, int Q, int C, int K, int st, int Nimg) {
  int nb, bpi;
  return hwg_plan(H, W, P, Q, C, K, st, Nimg, &nb, &bpi);
}

// ws: tfk_hwgrad_slabs(...) slabs of K*9*C f32. Returns -1 when the shape is not served, -2 on a
// launch error.
extern "C" int tfk_hwgrad_launch(const void* x, const void* dy, float* ws, int Nimg, int H, int W, int P, int Q, int C,
                                 int K, int st, int slabs, hipStream_t stream) {
  hwg::HWParams p;
  const int gx = hwg_plan(H, W, P, Q, C, K, st, Nimg, &p.nbands, &p.bands_per_img);
  if (gx < 1 || gx != slabs) return -1;
  p.x = (const bf16*)x;
  p.dy = (const bf16*)dy;
  p.ws = ws;
  p.Nimg = Nimg;
  p.H = H;
  p.W = W;
  p.P = P;
  p.C = C;
  p.K = K;
  p.slab = (long long)K * 9 * C;
  p.bands_per_block = (p.nbands + gx - 1) / gx;
  const dim3 grid(gx * (K / 64) * (C / 64)), block(512);
#define TFK_HWG(Q_, TR_, NB_, ST_)                                                                     \
  if (Q == Q_ && st == ST_) {                                                                          \
    hipLaunchKernelGGL((hwg::hwgrad_kernel<Q_, TR_, NB_, ST_>), grid, block, 0, stream, p);            \
    return hipGetLastError() == hipSuccess ? 0 : -2;                                                   \
  }
  TFK_HWG(56, 4, 1, 1)
  TFK_HWG(28, 7, 1, 1)
  TFK_HWG(14, 14, 1, 1)
  TFK_HWG(7, 7, 3, 1)
  TFK_HWG(28, 2, 1, 2)
  TFK_HWG(14, 7, 1, 2)
#undef TFK_HWG
  return -1;
}
