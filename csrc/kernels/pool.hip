// NHWC bf16 pooling for gfx950: max-pool (argmax byte recorded in forward, gather-form backward:
// no atomics) and global average pool. 8 channels (16 B) per lane.
#include "common.h"

namespace {
constexpr int NT = 256;

// bsc/bsh (optional): the pooled input is relu(x*bsc + bsh) of the producer's BatchNorm, applied
// here element by element (rounded to bf16 as the standalone BN pass stores it) -- the ResNet stem's
// BN output is read only by this pool, so it is never written (2 x 411 MB per bs-256 step).
__global__ void maxpool_fwd_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, uint8_t* __restrict__ idx, int N, int H,
                                   int W, int C, int P, int Q, int KH, int KW, int sh, int sw, int ph, int pw,
                                   const float* __restrict__ bsc, const float* __restrict__ bsh) {
  const int cpr = C >> 3;
  const long long total = (long long)N * P * Q * cpr;
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < total; i += (long long)gridDim.x * NT) {
    int cc = (int)(i % cpr);
    long long pix = i / cpr;
    int q = (int)(pix % Q);
    long long t = pix / Q;
    int p = (int)(t % P);
    int n = (int)(t / P);
    float best[8], sc[8], sf[8];
    uint8_t bi[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      best[e] = -INFINITY; bi[e] = 0;
      sc[e] = bsc ? bsc[cc * 8 + e] : 1.f;
      sf[e] = bsc ? bsh[cc * 8 + e] : 0.f;
    }
    for (int r = 0; r < KH; ++r) {
      int h = p * sh - ph + r;
      if ((unsigned)h >= (unsigned)H) continue;
      for (int s = 0; s < KW; ++s) {
        int w = q * sw - pw + s;
        if ((unsigned)w >= (unsigned)W) continue;
        bf16x8 v = *(const bf16x8*)(x + (((long long)n * H + h) * W + w) * C + cc * 8);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float f = bf2f(v[e]);
          if (bsc) f = bf2f(f2bf(fmaxf(f * sc[e] + sf[e], 0.f)));
          if (f > best[e]) { best[e] = f; bi[e] = (uint8_t)(r * KW + s); }
        }
      }
    }
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f2bf(best[e]);
    *(bf16x8*)(y + i * 8) = o;
    uint2 packed;
    packed.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | ((uint32_t)bi[3] << 24);
    packed.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | ((uint32_t)bi[7] << 24);
    *(uint2*)(idx + i * 8) = packed;
  }
}

// BNR: also accumulate the BN-backward channel sums of the layer that produced the pooled input
// (the ResNet stem), dz = dx * relu-mask: sums[shard][0][c] += dz, [1][c] += dz*(y-mean)*invstd --
// the standalone bn_bwd_reduce pass would re-read dx and y (846 MB at bs256). Mask: amask bit if
// given, else y*mscale+mshift > 0 if mscale is given, else 1. Needs NT % (C/8) == 0 (a thread's
// channel chunk is fixed across the grid-stride loop).
template <bool BNR>
__global__ void maxpool_bwd_kernel(const bf16* __restrict__ dy, const uint8_t* __restrict__ idx, bf16* __restrict__ dx, int N,
                                   int H, int W, int C, int P, int Q, int KH, int KW, int sh, int sw, int ph, int pw,
                                   const bf16* __restrict__ y, const float* __restrict__ mean,
                                   const float* __restrict__ invstd, const float* __restrict__ mscale,
                                   const float* __restrict__ mshift, const unsigned char* __restrict__ amask,
                                   float* __restrict__ sums, int shards) {
  const int cpr = C >> 3;
  const long long total = (long long)N * H * W * cpr;
  float s0[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s1[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  float mu[8], is[8], ms[8], mh[8];
  const int c0 = (threadIdx.x % cpr) * 8;
  if constexpr (BNR) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      mu[e] = mean[c0 + e]; is[e] = invstd[c0 + e];
      ms[e] = mscale ? mscale[c0 + e] : 1.f; mh[e] = mshift ? mshift[c0 + e] : 0.f;
    }
  }
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < total; i += (long long)gridDim.x * NT) {
    int cc = (int)(i % cpr);
    long long pix = i / cpr;
    int w = (int)(pix % W);
    long long t = pix / W;
    int h = (int)(t % H);
    int n = (int)(t / H);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    // outputs p with p*sh - ph <= h <= p*sh - ph + KH - 1
    int p_lo = (h + ph - KH + 1 + sh - 1) / sh; if (h + ph - KH + 1 < 0) p_lo = 0;
    int p_hi = (h + ph) / sh; if (p_hi > P - 1) p_hi = P - 1;
    int q_lo = (w + pw - KW + 1 + sw - 1) / sw; if (w + pw - KW + 1 < 0) q_lo = 0;
    int q_hi = (w + pw) / sw; if (q_hi > Q - 1) q_hi = Q - 1;
    for (int p = p_lo; p <= p_hi; ++p) {
      int r = h - (p * sh - ph);
      for (int q = q_lo; q <= q_hi; ++q) {
        int s = w - (q * sw - pw);
        uint8_t want = (uint8_t)(r * KW + s);
        long long o = (((long long)n * P + p) * Q + q) * C + cc * 8;
        bf16x8 g = *(const bf16x8*)(dy + o);
        uint2 packed = *(const uint2*)(idx + o);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          uint32_t word = e < 4 ? packed.x : packed.y;
          uint8_t b = (word >> (8 * (e & 3))) & 0xff;
          if (b == want) acc[e] += bf2f(g[e]);
        }
      }
    }
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f2bf(acc[e]);
    *(bf16x8*)(dx + i * 8) = o;
    if constexpr (BNR) {
      const bf16x8 yv = *(const bf16x8*)(y + i * 8);
      const unsigned mb = amask ? amask[i] : 0xffu;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float yf = bf2f(yv[e]);
        float dz = bf2f(o[e]);  // the stored (bf16-rounded) gradient, as the standalone pass reads it
        if (!((mb >> e) & 1u)) dz = 0.f;
        if (!amask && mscale && !(yf * ms[e] + mh[e] > 0.f)) dz = 0.f;
        s0[e] += dz;
        s1[e] += dz * (yf - mu[e]) * is[e];
      }
    }
  }
  if constexpr (BNR) {
    __shared__ float red[2][NT * 8];
    const int t = threadIdx.x;
#pragma unroll
    for (int e = 0; e < 8; ++e) { red[0][t * 8 + e] = s0[e]; red[1][t * 8 + e] = s1[e]; }
    __syncthreads();
    if (t < cpr) {
      float* st = sums + (long long)(blockIdx.x % shards) * 3 * C;
      for (int pass = 0; pass < 2; ++pass) {
        float a8[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) a8[e] = 0.f;
        for (int rr = t; rr < NT; rr += cpr)
#pragma unroll
          for (int e = 0; e < 8; ++e) a8[e] += red[pass][rr * 8 + e];
#pragma unroll
        for (int e = 0; e < 8; ++e) atomicAdd(st + pass * C + c0 + e, a8[e]);
      }
    }
  }
}

// 3x3 / stride 2 / pad 1 (the ResNet stem pool): an input row h is covered by output row h/2
// (even h) or rows (h-1)/2 and (h+1)/2 (odd h), likewise columns -- at most 4 windows, whose dy and
// argmax loads are ALL issued before any is used (the generic kernel's loop over the window range
// has one dependent load pair in flight per thread: latency-bound, 42 % of the HBM floor). BNR as
// in maxpool_bwd_kernel; the pixel's y is loaded with the windows.
template <bool BNR>
__global__ __launch_bounds__(NT) void maxpool_bwd_k3s2_kernel(
    const bf16* __restrict__ dy, const uint8_t* __restrict__ idx, bf16* __restrict__ dx, int N, int H, int W, int C,
    int P, int Q, const bf16* __restrict__ y, const float* __restrict__ mean, const float* __restrict__ invstd,
    const float* __restrict__ mscale, const float* __restrict__ mshift, const unsigned char* __restrict__ amask,
    float* __restrict__ sums, int shards) {
  const int cpr = C >> 3;
  const long long total = (long long)N * H * W * cpr;
  float s0[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s1[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  float mu[8], is[8], ms[8], mh[8];
  const int c0 = (threadIdx.x % cpr) * 8;
  if constexpr (BNR) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      mu[e] = mean[c0 + e]; is[e] = invstd[c0 + e];
      ms[e] = mscale ? mscale[c0 + e] : 1.f; mh[e] = mshift ? mshift[c0 + e] : 0.f;
    }
  }
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < total; i += (long long)gridDim.x * NT) {
    const int cc = (int)(i % cpr);
    const long long pix = i / cpr;
    const int w = (int)(pix % W);
    const long long t = pix / W;
    const int h = (int)(t % H);
    const int n = (int)(t / H);
    // candidate windows: rows pa = (h+1)/2 (always valid when < P), pb = (h-1)/2 (odd h only)
    const int pa = (h + 1) >> 1, pb = (h - 1) >> 1, qa = (w + 1) >> 1, qb = (w - 1) >> 1;
    const bool va = pa < P, vb = (h & 1) && pb >= 0, wa = qa < Q, wb = (w & 1) && qb >= 0;
    const int pr[2] = {va ? pa : 0, vb ? pb : 0}, qr[2] = {wa ? qa : 0, wb ? qb : 0};
    const bool vr[2] = {va, vb}, vc[2] = {wa, wb};
    bf16x8 g[4];
    uint2 id[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const long long o = (((long long)n * P + pr[k >> 1]) * Q + qr[k & 1]) * C + cc * 8;
      g[k] = *(const bf16x8*)(dy + o);
      id[k] = *(const uint2*)(idx + o);
    }
    bf16x8 yv;
    if constexpr (BNR) yv = *(const bf16x8*)(y + i * 8);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (!(vr[k >> 1] && vc[k & 1])) continue;
      const int r = h - (pr[k >> 1] * 2 - 1), sc = w - (qr[k & 1] * 2 - 1);
      const uint8_t want = (uint8_t)(r * 3 + sc);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const uint32_t word = e < 4 ? id[k].x : id[k].y;
        if (((word >> (8 * (e & 3))) & 0xff) == want) acc[e] += bf2f(g[k][e]);
      }
    }
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f2bf(acc[e]);
    *(bf16x8*)(dx + i * 8) = o;
    if constexpr (BNR) {
      const unsigned mb = amask ? amask[i] : 0xffu;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float yf = bf2f(yv[e]);
        float dz = bf2f(o[e]);
        if (!((mb >> e) & 1u)) dz = 0.f;
        if (!amask && mscale && !(yf * ms[e] + mh[e] > 0.f)) dz = 0.f;
        s0[e] += dz;
        s1[e] += dz * (yf - mu[e]) * is[e];
      }
    }
  }
  if constexpr (BNR) {
    __shared__ float red[2][NT * 8];
    const int t = threadIdx.x;
#pragma unroll
    for (int e = 0; e < 8; ++e) { red[0][t * 8 + e] = s0[e]; red[1][t * 8 + e] = s1[e]; }
    __syncthreads();
    if (t < cpr) {
      float* st = sums + (long long)(blockIdx.x % shards) * 3 * C;
      for (int pass = 0; pass < 2; ++pass) {
        float a8[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) a8[e] = 0.f;
        for (int rr = t; rr < NT; rr += cpr)
#pragma unroll
          for (int e = 0; e < 8; ++e) a8[e] += red[pass][rr * 8 + e];
#pragma unroll
        for (int e = 0; e < 8; ++e) atomicAdd(st + pass * C + c0 + e, a8[e]);
      }
    }
  }
}

// x [N][HW][C] -> y [N][C] (bf16), mean over HW. One block per (n, 8*NT channel slab).
__global__ void avgpool_fwd_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, int HW, int C) {
  const int n = blockIdx.y;
  const int c = (blockIdx.x * NT + threadIdx.x) * 8;
  if (c >= C) return;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const bf16* base = x + (long long)n * HW * C + c;
  for (int i = 0; i < HW; ++i) {
    bf16x8 v = *(const bf16x8*)(base + (long long)i * C);
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] += bf2f(v[e]);
  }
  bf16x8 o;
  const float inv = 1.f / HW;
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = f2bf(acc[e] * inv);
  *(bf16x8*)(y + (long long)n * C + c) = o;
}

__global__ void avgpool_bwd_kernel(const bf16* __restrict__ dy, bf16* __restrict__ dx, int N, int HW, int C) {
  const int cpr = C >> 3;
  const long long total = (long long)N * HW * cpr;
  const float inv = 1.f / HW;
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < total; i += (long long)gridDim.x * NT) {
    int cc = (int)(i % cpr);
    long long n = i / cpr / HW;
    bf16x8 g = *(const bf16x8*)(dy + n * C + cc * 8);
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f2bf(bf2f(g[e]) * inv);
    *(bf16x8*)(dx + i * 8) = o;
  }
}

int grid_for(long long work, int cap = 8192) {
  long long g = (work + NT - 1) / NT;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}
}  // namespace

extern "C" {
int tfk_maxpool_fwd(const bf16* x, bf16* y, uint8_t* idx, int N, int H, int W, int C, int P, int Q, int KH, int KW, int sh,
                    int sw, int ph, int pw, const float* bsc, const float* bsh, hipStream_t s) {
  long long total = (long long)N * P * Q * (C / 8);
  hipLaunchKernelGGL(maxpool_fwd_kernel, dim3(grid_for(total)), dim3(NT), 0, s, x, y, idx, N, H, W, C, P, Q, KH, KW, sh, sw,
                     ph, pw, bsc, bsh);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int tfk_maxpool_bwd(const bf16* dy, const uint8_t* idx, bf16* dx, int N, int H, int W, int C, int P, int Q, int KH, int KW,
                    int sh, int sw, int ph, int pw, const bf16* y, const float* mean, const float* invstd,
                    const float* mscale, const float* mshift, const unsigned char* amask, float* sums, int shards,
                    hipStream_t s) {
  long long total = (long long)N * H * W * (C / 8);
  if (KH == 3 && KW == 3 && sh == 2 && sw == 2 && ph == 1 && pw == 1 && NT % (C / 8) == 0 &&
      P == (H - 1) / 2 + 1 && Q == (W - 1) / 2 + 1) {
    if (sums) {
      if (shards < 1) return -1;
      hipLaunchKernelGGL(maxpool_bwd_k3s2_kernel<true>, dim3(grid_for(total)), dim3(NT), 0, s, dy, idx, dx, N, H, W, C, P,
                         Q, y, mean, invstd, mscale, mshift, amask, sums, shards);
    } else {
      hipLaunchKernelGGL(maxpool_bwd_k3s2_kernel<false>, dim3(grid_for(total)), dim3(NT), 0, s, dy, idx, dx, N, H, W, C,
                         P, Q, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 1);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
  if (sums) {
    if (NT % (C / 8) != 0 || shards < 1) return -1;
    hipLaunchKernelGGL(maxpool_bwd_kernel<true>, dim3(grid_for(total)), dim3(NT), 0, s, dy, idx, dx, N, H, W, C, P, Q, KH,
                       KW, sh, sw, ph, pw, y, mean, invstd, mscale, mshift, amask, sums, shards);
  } else {
    hipLaunchKernelGGL(maxpool_bwd_kernel<false>, dim3(grid_for(total)), dim3(NT), 0, s, dy, idx, dx, N, H, W, C, P, Q, KH,
                       KW, sh, sw, ph, pw, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 1);
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int tfk_avgpool_fwd(const bf16* x, bf16* y, int N, int HW, int C, hipStream_t s) {
  dim3 grid((C / 8 + NT - 1) / NT, N);
  hipLaunchKernelGGL(avgpool_fwd_kernel, grid, dim3(NT), 0, s, x, y, HW, C);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int tfk_avgpool_bwd(const bf16* dy, bf16* dx, int N, int HW, int C, hipStream_t s) {
  long long total = (long long)N * HW * (C / 8);
  hipLaunchKernelGGL(avgpool_bwd_kernel, dim3(grid_for(total)), dim3(NT), 0, s, dy, dx, N, HW, C);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
}
