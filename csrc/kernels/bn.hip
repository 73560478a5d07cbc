// Training-mode BatchNorm for NHWC bf16 activations [M = N*H*W][C], C % 8 == 0.
//
// Forward statistics are accumulated by the producing conv's GEMM epilogue (gemm.hip, sharded
// f32 atomics), so the forward here is: finalize (shards -> mean/invstd/scale/shift, running
// stats) + one fused apply pass  a = relu(y*scale + shift [+ r | + r*rscale + rshift]).
// The dual-input form fuses a projection shortcut's BN into the residual add of the block.
// Backward: reduce (sum dz, sum dz*xhat[, sum dz*xhat2]) -> finalize (dgamma/dbeta + apply
// coefficients) -> apply (dy[, dy2 | dres]), where dz = da * 1[a > 0].
#include "common.h"
#include "bn_fin.h"

#include <algorithm>

namespace {
using tfk::BnFin;
using tfk::BnBwdFin;
constexpr int NT = 256;
constexpr int SHARD_UNROLL = 4;  // shards <= 16 (ops/norm.py SHARDS): loads per thread issued together

// ---------------------------------------------------------------- forward
// Sums NV per-channel vectors stored as [shards][NV][C] over the shards for channel c, zeroing the
// shards for the next accumulation. 256-thread blocks = 64 channels x 4 shard groups: each thread
// issues shards/4 independent loads (latency-bound otherwise), then a 4-way LDS reduction.
template <int NV>
__device__ __forceinline__ bool shard_sum(float* buf, int shards, int C, float (&out)[NV]) {
  __shared__ float red[4][NV][64];
  const int l = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + l;
  float acc[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) acc[v] = 0.f;
  if (c < C) {
    if (shards <= 4 * SHARD_UNROLL) {
      // every load of this thread's shards issued before any is used (clamped shard index, masked
      // contribution): one memory latency instead of shards/4 chained ones -- the finalize kernels
      // sit on the critical path between a conv and its BN apply
      float x[SHARD_UNROLL][NV];
#pragma unroll
      for (int k = 0; k < SHARD_UNROLL; ++k) {
        const int i = min(g + 4 * k, shards - 1);
        const float* p = buf + (long long)i * NV * C;
#pragma unroll
        for (int v = 0; v < NV; ++v) x[k][v] = p[v * C + c];
      }
#pragma unroll
      for (int k = 0; k < SHARD_UNROLL; ++k)
#pragma unroll
        for (int v = 0; v < NV; ++v) acc[v] += g + 4 * k < shards ? x[k][v] : 0.f;
    } else {
      for (int i = g; i < shards; i += 4) {
        float* p = buf + (long long)i * NV * C;
#pragma unroll
        for (int v = 0; v < NV; ++v) acc[v] += p[v * C + c];
      }
    }
    for (int i = g; i < shards; i += 4) {
      float* p = buf + (long long)i * NV * C;
#pragma unroll
      for (int v = 0; v < NV; ++v) p[v * C + c] = 0.f;
    }
  }
#pragma unroll
  for (int v = 0; v < NV; ++v) red[g][v][l] = acc[v];
  __syncthreads();
  if (g != 0 || c >= C) return false;
#pragma unroll
  for (int v = 0; v < NV; ++v) out[v] = red[0][v][l] + red[1][v][l] + red[2][v][l] + red[3][v][l];
  return true;
}

// stats: [shards][2][C] (sum, sumsq), zeroed again after reading so the next conv can accumulate.
__global__ __launch_bounds__(256) void bn_finalize_kernel(float* stats, int shards, int C, float count,
                                                          const float* __restrict__ gamma, const float* __restrict__ beta,
                                                          float eps, float momentum, float* __restrict__ run_mean,
                                                          float* __restrict__ run_var, float* __restrict__ mean_out,
                                                          float* __restrict__ invstd_out, float* __restrict__ scale_out,
                                                          float* __restrict__ shift_out) {
  float sq[2];
  if (!shard_sum<2>(stats, shards, C, sq)) return;
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const float s = sq[0], q = sq[1];
  double mean = (double)s / count;
  double var = (double)q / count - mean * mean;
  if (var < 0) var = 0;
  float inv = rsqrtf((float)var + eps);
  mean_out[c] = (float)mean;
  invstd_out[c] = inv;
  float g = gamma[c], b = beta[c];
  scale_out[c] = g * inv;
  shift_out[c] = b - (float)mean * g * inv;
  if (run_mean) {
    float unb = count > 1.f ? (float)var * count / (count - 1.f) : (float)var;
    run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * (float)mean;
    run_var[c] = (1.f - momentum) * run_var[c] + momentum * unb;
  }
}

// Plain statistics pass for tensors that did not come out of a GEMM epilogue.
__global__ void bn_stats_kernel(const bf16* __restrict__ y, long long M, int C, float* __restrict__ stats, int shards) {
  const int cpr = C >> 3;                 // 8-channel chunks per row
  const int rows_par = NT / cpr > 0 ? NT / cpr : 1;
  const int t = threadIdx.x;
  const int cchunk = t % cpr, rsub = t / cpr;
  float s[8] = {0}, q[8] = {0};
  if (rsub < rows_par) {
    for (long long r = (long long)blockIdx.x * rows_par + rsub; r < M; r += (long long)gridDim.x * rows_par) {
      bf16x8 v = *(const bf16x8*)(y + r * C + cchunk * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) { float x = bf2f(v[e]); s[e] += x; q[e] += x * x; }
    }
  }
  __shared__ float red[NT * 8];
  float* st = stats + (long long)(blockIdx.x % shards) * 2 * C;
  for (int pass = 0; pass < 2; ++pass) {
    float* src = pass ? q : s;
    __syncthreads();
#pragma unroll
    for (int e = 0; e < 8; ++e) red[t * 8 + e] = src[e];
    __syncthreads();
    if (rsub == 0) {
      for (int rr = 1; rr < rows_par; ++rr)
#pragma unroll
        for (int e = 0; e < 8; ++e) src[e] += red[(rr * cpr + cchunk) * 8 + e];
#pragma unroll
      for (int e = 0; e < 8; ++e) atomicAdd(st + pass * C + cchunk * 8 + e, src[e]);
    }
  }
}

__device__ __forceinline__ void load8(const float* __restrict__ p, float (&v)[8]) {
  f32x4 a = *(const f32x4*)p, b = *(const f32x4*)(p + 4);
#pragma unroll
  for (int e = 0; e < 4; ++e) { v[e] = a[e]; v[e + 4] = b[e]; }
}

// Streaming passes: with FIXED a thread owns one 8-channel chunk (tid % cpr) and walks rows, so
// per-channel coefficients are loaded once into registers; needs NT % cpr == 0 (C | 2048). Other
// C use the flat layout and reload the chunk's coefficients per element group.
template <bool FIXED>
__global__ __launch_bounds__(NT) void bn_apply_kernel(const bf16* __restrict__ y, const float* __restrict__ scale, const float* __restrict__ shift,
                                const bf16* __restrict__ r, const float* __restrict__ rscale, const float* __restrict__ rshift,
                                int relu, bf16* __restrict__ out, long long M, int C, unsigned char* __restrict__ mask) {
  const int cpr = C >> 3;
  long long i, step;
  int c0;
  if (FIXED) {
    const int rows_par = NT / cpr;
    c0 = (threadIdx.x % cpr) * 8;
    i = ((long long)blockIdx.x * rows_par + threadIdx.x / cpr) * C + c0;
    step = (long long)gridDim.x * rows_par * C;
  } else {
    i = ((long long)blockIdx.x * NT + threadIdx.x) * 8;
    step = (long long)gridDim.x * NT * 8;
    c0 = 0;
  }
  const long long end = M * C;
  float s[8], b[8], rs[8], rb[8];
  if (FIXED) {
    load8(scale + c0, s); load8(shift + c0, b);
    if (rscale) { load8(rscale + c0, rs); load8(rshift + c0, rb); }
  }
  for (; i < end; i += step) {
    if (!FIXED) {
      c0 = (int)((i >> 3) % cpr) * 8;
      load8(scale + c0, s); load8(shift + c0, b);
      if (rscale) { load8(rscale + c0, rs); load8(rshift + c0, rb); }
    }
    bf16x8 v = *(const bf16x8*)(y + i);
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = bf2f(v[e]) * s[e] + b[e];
    if (r) {
      bf16x8 rv = *(const bf16x8*)(r + i);
      if (rscale) {
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] += bf2f(rv[e]) * rs[e] + rb[e];
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] += bf2f(rv[e]);
      }
    }
    bf16x8 w;
#pragma unroll
    for (int e = 0; e < 8; ++e) w[e] = f2bf(relu ? fmaxf(o[e], 0.f) : o[e]);
    *(bf16x8*)(out + i) = w;
    if (mask) {
      // bit e of byte i/8 = (out[i+e] > 0): the backward's relu mask at 1/16 of out's bytes
      unsigned bits = 0;
#pragma unroll
      for (int e = 0; e < 8; ++e) bits |= (bf2f(w[e]) > 0.f ? 1u : 0u) << e;
      mask[i >> 3] = (unsigned char)bits;
    }
  }
}

// ---------------------------------------------------------------- backward
// sums: [shards][3][C]: sum dz, sum dz*xhat, sum dz*xhat2
__global__ void bn_bwd_reduce_kernel(const bf16* __restrict__ da, const bf16* __restrict__ a, const bf16* __restrict__ y,
                                     const float* __restrict__ mean, const float* __restrict__ invstd,
                                     const bf16* __restrict__ y2, const float* __restrict__ mean2,
                                     const float* __restrict__ invstd2, long long M, int C, float* __restrict__ sums,
                                     int shards, const float* __restrict__ mscale, const float* __restrict__ mshift,
                                     const unsigned char* __restrict__ amask) {
  const int cpr = C >> 3;
  const int rows_par = NT / cpr > 0 ? NT / cpr : 1;
  const int t = threadIdx.x;
  const int cchunk = t % cpr, rsub = t / cpr;
  const int c0 = cchunk * 8;
  float s0[8] = {0}, s1[8] = {0}, s2[8] = {0};
  if (rsub < rows_par) {
    float mu[8], is[8], mu2[8], is2[8], msc[8], msh[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      mu[e] = mean[c0 + e]; is[e] = invstd[c0 + e];
      msc[e] = mscale ? mscale[c0 + e] : 1.f; msh[e] = mshift ? mshift[c0 + e] : 0.f;
      mu2[e] = y2 ? mean2[c0 + e] : 0.f; is2[e] = y2 ? invstd2[c0 + e] : 0.f;
    }
    for (long long r = (long long)blockIdx.x * rows_par + rsub; r < M; r += (long long)gridDim.x * rows_par) {
      const long long off = r * C + c0;
      bf16x8 g = *(const bf16x8*)(da + off);
      bf16x8 yv = *(const bf16x8*)(y + off);
      bf16x8 av;
      if (a) av = *(const bf16x8*)(a + off);
      const unsigned mb = amask ? amask[off >> 3] : 0xffu;
      bf16x8 y2v;
      if (y2) y2v = *(const bf16x8*)(y2 + off);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float dz = bf2f(g[e]);
        if (!((mb >> e) & 1u)) dz = 0.f;
        if (a && !(bf2f(av[e]) > 0.f)) dz = 0.f;
        if (!a && mscale && !(bf2f(yv[e]) * msc[e] + msh[e] > 0.f)) dz = 0.f;
        s0[e] += dz;
        s1[e] += dz * (bf2f(yv[e]) - mu[e]) * is[e];
        if (y2) s2[e] += dz * (bf2f(y2v[e]) - mu2[e]) * is2[e];
      }
    }
  }
  // all three partial vectors to LDS at once (a pointer selecting between local arrays would put
  // them in scratch)
  __shared__ float red[3][NT * 8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { red[0][t * 8 + e] = s0[e]; red[1][t * 8 + e] = s1[e]; red[2][t * 8 + e] = s2[e]; }
  __syncthreads();
  if (rsub == 0) {
    float* st = sums + (long long)(blockIdx.x % shards) * 3 * C;
    const int npass = y2 ? 3 : 2;
    for (int pass = 0; pass < npass; ++pass) {
      float acc[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] = red[pass][cchunk * 8 + e];
      for (int rr = 1; rr < rows_par; ++rr)
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += red[pass][(rr * cpr + cchunk) * 8 + e];
#pragma unroll
      for (int e = 0; e < 8; ++e) atomicAdd(st + pass * C + c0 + e, acc[e]);
    }
  }
}

// Reduce shards; write dgamma/dbeta (+= if accumulate) and per-channel apply coefficients.
// With k1 = gamma*invstd, dy = k1*(dz - mean(dz) - xhat*mean(dz*xhat)) is affine in (dz, y):
// coef = [k1, A, B][C] with dy = k1*dz + A*y + B; coef2 the same for the second BN.
__global__ __launch_bounds__(256) void bn_bwd_finalize_kernel(float* sums, int shards, int C, float count,
                                       const float* __restrict__ gamma, const float* __restrict__ mean,
                                       const float* __restrict__ invstd, const float* __restrict__ gamma2,
                                       const float* __restrict__ mean2, const float* __restrict__ invstd2,
                                       float* __restrict__ dgamma, float* __restrict__ dbeta, float* __restrict__ dgamma2,
                                       float* __restrict__ dbeta2, float* __restrict__ coef, float* __restrict__ coef2) {
  float sv[3];
  if (!shard_sum<3>(sums, shards, C, sv)) return;
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const float s0 = sv[0], s1 = sv[1], s2 = sv[2];
  dgamma[c] = s1;
  dbeta[c] = s0;
  {
    const float inv = invstd[c], k1 = gamma[c] * inv, k3 = s1 / count;
    coef[c] = k1;
    coef[C + c] = -k1 * k3 * inv;
    coef[2 * C + c] = k1 * (k3 * inv * mean[c] - s0 / count);
  }
  if (coef2) {
    dgamma2[c] = s2;
    dbeta2[c] = s0;
    const float inv = invstd2[c], k1 = gamma2[c] * inv, k3 = s2 / count;
    coef2[c] = k1;
    coef2[C + c] = -k1 * k3 * inv;
    coef2[2 * C + c] = k1 * (k3 * inv * mean2[c] - s0 / count);
  }
}

// dy = k1*dz + A*y + B; optional dy2 (projection-shortcut BN) or dres = dz (identity shortcut).
// Relu mask: a > 0 if a is given, else y*mscale + mshift > 0 if mscale is given, else none.
template <bool FIXED>
__global__ __launch_bounds__(NT) void bn_bwd_apply_kernel(const bf16* __restrict__ da, const bf16* __restrict__ a, const bf16* __restrict__ y,
                                    const float* __restrict__ coef, bf16* __restrict__ dy, const bf16* __restrict__ y2,
                                    const float* __restrict__ coef2, bf16* __restrict__ dy2, bf16* __restrict__ dres,
                                    long long M, int C, const float* __restrict__ mscale,
                                    const float* __restrict__ mshift, const unsigned char* __restrict__ amask) {
  const int cpr = C >> 3;
  long long i, step;
  int c0;
  if (FIXED) {
    const int rows_par = NT / cpr;
    c0 = (threadIdx.x % cpr) * 8;
    i = ((long long)blockIdx.x * rows_par + threadIdx.x / cpr) * C + c0;
    step = (long long)gridDim.x * rows_par * C;
  } else {
    i = ((long long)blockIdx.x * NT + threadIdx.x) * 8;
    step = (long long)gridDim.x * NT * 8;
    c0 = 0;
  }
  const long long end = M * C;
  float k1[8], A[8], B[8], k1b[8], A2[8], B2[8], ms[8], mh[8];
  auto load_coefs = [&]() {
    load8(coef + c0, k1); load8(coef + C + c0, A); load8(coef + 2 * C + c0, B);
    if (y2) { load8(coef2 + c0, k1b); load8(coef2 + C + c0, A2); load8(coef2 + 2 * C + c0, B2); }
    if (!a && mscale) { load8(mscale + c0, ms); load8(mshift + c0, mh); }
  };
  if (FIXED) load_coefs();
  for (; i < end; i += step) {
    if (!FIXED) {
      c0 = (int)((i >> 3) % cpr) * 8;
      load_coefs();
    }
    bf16x8 g = *(const bf16x8*)(da + i);
    bf16x8 yv = *(const bf16x8*)(y + i);
    bf16x8 av;
    if (a) av = *(const bf16x8*)(a + i);
    const unsigned mb = amask ? amask[i >> 3] : 0xffu;
    float dz[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      dz[e] = bf2f(g[e]);
      if (amask) {
        if (!((mb >> e) & 1u)) dz[e] = 0.f;
      } else if (a) {
        if (!(bf2f(av[e]) > 0.f)) dz[e] = 0.f;
      } else if (mscale) {
        if (!(bf2f(yv[e]) * ms[e] + mh[e] > 0.f)) dz[e] = 0.f;
      }
    }
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f2bf(k1[e] * dz[e] + A[e] * bf2f(yv[e]) + B[e]);
    *(bf16x8*)(dy + i) = o;
    if (y2) {
      bf16x8 y2v = *(const bf16x8*)(y2 + i);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = f2bf(k1b[e] * dz[e] + A2[e] * bf2f(y2v[e]) + B2[e]);
      *(bf16x8*)(dy2 + i) = o;
    }
    if (dres) {
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = f2bf(dz[e]);
      *(bf16x8*)(dres + i) = o;
    }
  }
}

// ---------------------------------------------------------------- finalize folded into apply
// The separate finalize launches sat on the critical path between each conv and its BN pass
// (ResNet-50 bs256: skipping all 102 of them measured 0.71 ms/step, profiles/perf_log_r5.md). Here
// every apply block finalizes the 64-channel slice it streams: it reduces the slice's shard
// partials (L2-resident: the producing GEMM's atomics just wrote them) into LDS, derives its
// coefficients, and row group 0 of the slice writes the saved statistics / running stats /
// parameter gradients. The shards are NOT zeroed here (every block of the slice reads them): the
// owning model zeroes all pooled BN accumulators once per step (tfk_bn_zero, ops/norm.py BNPool).
// Grid: x = C/64 channel slices, y = row groups; block = 8 chunk lanes x 32 rows.
constexpr int FIN_SHARDS = 16;  // pooled states (ops/norm.py SHARDS)


// Sum [shards][NV][C] over the shards for channels c0..c0+63 into tot[NV][64] (LDS). All threads.
template <int NV>
__device__ __forceinline__ void slice_sum(const float* __restrict__ buf, int shards, int C, int c0,
                                          float (*part)[NV][64], float (*tot)[64]) {
  const int t = threadIdx.x;
  for (int q = t; q < FIN_SHARDS * NV * 8; q += NT) {
    const int i = q / (NV * 8), rem = q - i * NV * 8, v = rem >> 3, ch = rem & 7;
    float x[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (i < shards) load8(buf + ((long long)i * NV + v) * C + c0 + ch * 8, x);
#pragma unroll
    for (int e = 0; e < 8; ++e) part[i][v][ch * 8 + e] = x[e];
  }
  __syncthreads();
  if (t < NV * 64) {
    const int v = t >> 6, c = t & 63;
    float a = 0.f;
#pragma unroll
    for (int i = 0; i < FIN_SHARDS; ++i) a += part[i][v][c];
    tot[v][c] = a;
  }
  __syncthreads();
}

// Forward finalize of channel slice c0 into sc/sh (LDS); row group 0 publishes the statistics.
__device__ __forceinline__ void fin_fwd(const BnFin& f, int C, int c0, float count, float (*part)[2][64],
                                        float (*tot)[64], float* sc, float* sh) {
  if (f.stats == nullptr) {
    if (threadIdx.x < 64) {
      sc[threadIdx.x] = f.scale[c0 + threadIdx.x];
      sh[threadIdx.x] = f.shift[c0 + threadIdx.x];
    }
    return;
  }
  slice_sum<2>(f.stats, f.shards, C, c0, part, tot);
  if (threadIdx.x < 64) {
    const int c = c0 + threadIdx.x;
    const double mean = (double)tot[0][threadIdx.x] / count;
    double var = (double)tot[1][threadIdx.x] / count - mean * mean;
    if (var < 0) var = 0;
    const float inv = rsqrtf((float)var + f.eps);
    const float g = f.gamma[c], b = f.beta[c];
    const float scale = g * inv, shift = b - (float)mean * g * inv;
    sc[threadIdx.x] = scale;
    sh[threadIdx.x] = shift;
    if (blockIdx.y == 0) {
      f.mean[c] = (float)mean;
      f.invstd[c] = inv;
      f.scale[c] = scale;
      f.shift[c] = shift;
      if (f.run_mean) {
        const float unb = count > 1.f ? (float)var * count / (count - 1.f) : (float)var;
        f.run_mean[c] = (1.f - f.momentum) * f.run_mean[c] + f.momentum * (float)mean;
        f.run_var[c] = (1.f - f.momentum) * f.run_var[c] + f.momentum * unb;
      }
    }
  }
}

constexpr int FIN_ROWS = 4;  // rows per thread per iteration (loads issued together)

__global__ __launch_bounds__(256) void bn_apply_fin_kernel(const bf16* __restrict__ y, BnFin f, const bf16* __restrict__ r,
                                                           BnFin f2, int dual, int relu, bf16* __restrict__ out,
                                                           long long M, int C, unsigned char* __restrict__ mask,
                                                           long long rows_per_block) {
  __shared__ float part[FIN_SHARDS][2][64];
  __shared__ float tot[2][64];
  __shared__ float sc[2][64], sh[2][64];
  const int c0 = blockIdx.x * 64;
  const float count = (float)M;
  fin_fwd(f, C, c0, count, part, tot, sc[0], sh[0]);
  if (dual) {
    __syncthreads();
    fin_fwd(f2, C, c0, count, part, tot, sc[1], sh[1]);
  }
  __syncthreads();
  const int ch = threadIdx.x & 7, rsub = threadIdx.x >> 3;
  float s[8], b[8], rs[8], rb[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    s[e] = sc[0][ch * 8 + e]; b[e] = sh[0][ch * 8 + e];
    rs[e] = dual ? sc[1][ch * 8 + e] : 0.f; rb[e] = dual ? sh[1][ch * 8 + e] : 0.f;
  }
  const long long r0 = (long long)blockIdx.y * rows_per_block, r1 = min(M, r0 + rows_per_block);
  const int cc = c0 + ch * 8;
  for (long long base = r0 + rsub; base < r1; base += 32 * FIN_ROWS) {
    bf16x8 v[FIN_ROWS], rv[FIN_ROWS];
#pragma unroll
    for (int k = 0; k < FIN_ROWS; ++k) {
      const long long row = base + 32 * k;
      if (row < r1) {
        v[k] = *(const bf16x8*)(y + row * C + cc);
        if (r) rv[k] = *(const bf16x8*)(r + row * C + cc);
      }
    }
#pragma unroll
    for (int k = 0; k < FIN_ROWS; ++k) {
      const long long row = base + 32 * k;
      if (row >= r1) break;
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = bf2f(v[k][e]) * s[e] + b[e];
      if (r) {
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] += dual ? bf2f(rv[k][e]) * rs[e] + rb[e] : bf2f(rv[k][e]);
      }
      bf16x8 w;
#pragma unroll
      for (int e = 0; e < 8; ++e) w[e] = f2bf(relu ? fmaxf(o[e], 0.f) : o[e]);
      const long long i = row * C + cc;
      *(bf16x8*)(out + i) = w;
      if (mask) {
        unsigned bits = 0;
#pragma unroll
        for (int e = 0; e < 8; ++e) bits |= (bf2f(w[e]) > 0.f ? 1u : 0u) << e;
        mask[i >> 3] = (unsigned char)bits;
      }
    }
  }
}


__global__ __launch_bounds__(256) void bn_bwd_apply_fin_kernel(const bf16* __restrict__ da, const bf16* __restrict__ y,
                                                               const float* __restrict__ sums, int shards, BnBwdFin f,
                                                               const bf16* __restrict__ y2, BnBwdFin f2,
                                                               bf16* __restrict__ dy, bf16* __restrict__ dy2,
                                                               bf16* __restrict__ dres, long long M, int C,
                                                               const float* __restrict__ mscale,
                                                               const float* __restrict__ mshift,
                                                               const unsigned char* __restrict__ amask,
                                                               long long rows_per_block) {
  __shared__ float part[FIN_SHARDS][3][64];
  __shared__ float tot[3][64];
  __shared__ float cf[6][64];  // k1, A, B (, k1b, A2, B2)
  const int c0 = blockIdx.x * 64;
  const float count = (float)M;
  slice_sum<3>(sums, shards, C, c0, part, tot);
  if (threadIdx.x < 64) {
    const int l = threadIdx.x, c = c0 + l;
    const float s0 = tot[0][l], s1 = tot[1][l], s2 = tot[2][l];
    {
      const float inv = f.invstd[c], k1 = f.gamma[c] * inv, k3 = s1 / count;
      cf[0][l] = k1;
      cf[1][l] = -k1 * k3 * inv;
      cf[2][l] = k1 * (k3 * inv * f.mean[c] - s0 / count);
    }
    if (y2) {
      const float inv = f2.invstd[c], k1 = f2.gamma[c] * inv, k3 = s2 / count;
      cf[3][l] = k1;
      cf[4][l] = -k1 * k3 * inv;
      cf[5][l] = k1 * (k3 * inv * f2.mean[c] - s0 / count);
    }
    if (blockIdx.y == 0) {
      f.dgamma[c] = s1;
      f.dbeta[c] = s0;
      if (y2) { f2.dgamma[c] = s2; f2.dbeta[c] = s0; }
    }
  }
  __syncthreads();
  const int ch = threadIdx.x & 7, rsub = threadIdx.x >> 3;
  const int cc = c0 + ch * 8;
  float k1[8], A[8], B[8], k1b[8], A2[8], B2[8], ms[8], mh[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    k1[e] = cf[0][ch * 8 + e]; A[e] = cf[1][ch * 8 + e]; B[e] = cf[2][ch * 8 + e];
    k1b[e] = y2 ? cf[3][ch * 8 + e] : 0.f; A2[e] = y2 ? cf[4][ch * 8 + e] : 0.f; B2[e] = y2 ? cf[5][ch * 8 + e] : 0.f;
  }
  if (mscale) { load8(mscale + cc, ms); load8(mshift + cc, mh); }
  const long long r0 = (long long)blockIdx.y * rows_per_block, r1 = min(M, r0 + rows_per_block);
  for (long long base = r0 + rsub; base < r1; base += 32 * FIN_ROWS) {
    bf16x8 g[FIN_ROWS], yv[FIN_ROWS], y2v[FIN_ROWS];
    unsigned mb[FIN_ROWS];
#pragma unroll
    for (int k = 0; k < FIN_ROWS; ++k) {
      const long long row = base + 32 * k;
      if (row < r1) {
        const long long i = row * C + cc;
        g[k] = *(const bf16x8*)(da + i);
        yv[k] = *(const bf16x8*)(y + i);
        if (y2) y2v[k] = *(const bf16x8*)(y2 + i);
        mb[k] = amask ? amask[i >> 3] : 0xffu;
      }
    }
#pragma unroll
    for (int k = 0; k < FIN_ROWS; ++k) {
      const long long row = base + 32 * k;
      if (row >= r1) break;
      const long long i = row * C + cc;
      float dz[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        dz[e] = bf2f(g[k][e]);
        if (amask) {
          if (!((mb[k] >> e) & 1u)) dz[e] = 0.f;
        } else if (mscale) {
          if (!(bf2f(yv[k][e]) * ms[e] + mh[e] > 0.f)) dz[e] = 0.f;
        }
      }
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = f2bf(k1[e] * dz[e] + A[e] * bf2f(yv[k][e]) + B[e]);
      *(bf16x8*)(dy + i) = o;
      if (y2) {
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = f2bf(k1b[e] * dz[e] + A2[e] * bf2f(y2v[k][e]) + B2[e]);
        *(bf16x8*)(dy2 + i) = o;
      }
      if (dres) {
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = f2bf(dz[e]);
        *(bf16x8*)(dres + i) = o;
      }
    }
  }
}

__global__ void bn_zero_kernel(float* __restrict__ p, long long n) {
  const long long i = ((long long)blockIdx.x * NT + threadIdx.x) * 4;
  if (i + 3 < n) *(f32x4*)(p + i) = f32x4{0.f, 0.f, 0.f, 0.f};
  else
    for (long long k = i; k < n; ++k) p[k] = 0.f;
}

// Grid of the slice kernels: C/64 x row groups, ~FIN_BLOCKS blocks, >= 256 rows (8 row iterations of
// 32) per block so the finalize prologue amortizes.
constexpr int FIN_BLOCKS = 4096;
static dim3 fin_grid(long long M, int C, long long* rows_per_block) {
  const int slices = C / 64;
  long long groups = std::max(1LL, std::min<long long>((M + 255) / 256, FIN_BLOCKS / slices));
  long long rpb = (M + groups - 1) / groups;
  rpb = (rpb + 31) / 32 * 32;
  groups = (M + rpb - 1) / rpb;
  *rows_per_block = rpb;
  return dim3(slices, (unsigned)groups);
}

int grid_for(long long work, int per_block, int cap = 4096) {
  long long g = (work + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}
// Measurement probe only (tools/bench_with.py --set bn_fin_skip=N): 1 skips the forward finalize
// launches, 2 the backward ones, 3 both -- the step time then bounds what fusing them into the
// producing GEMM can save. Numerics are wrong while it is set.
int g_fin_skip = 0;
}  // namespace

extern "C" {
void tfk_bn_fin_skip(int v) { g_fin_skip = v; }
int tfk_bn_finalize(float* stats, int shards, int C, float count, const float* gamma, const float* beta, float eps,
                    float momentum, float* run_mean, float* run_var, float* mean, float* invstd, float* scale,
                    float* shift, hipStream_t s) {
  if (g_fin_skip & 1) return 0;
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + 63) / 64), dim3(256), 0, s, stats, shards, C, count, gamma, beta, eps,
                     momentum, run_mean, run_var, mean, invstd, scale, shift);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int tfk_bn_stats(const bf16* y, long long M, int C, float* stats, int shards, hipStream_t s) {
  int cpr = C / 8, rows_par = NT / cpr > 0 ? NT / cpr : 1;
  hipLaunchKernelGGL(bn_stats_kernel, dim3(grid_for(M, rows_par * 16, 2048)), dim3(NT), 0, s, y, M, C, stats, shards);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int tfk_bn_apply(const bf16* y, const float* scale, const float* shift, const bf16* r, const float* rscale,
                 const float* rshift, int relu, bf16* out, long long M, int C, unsigned char* mask, hipStream_t s) {
  const int cpr = C / 8;
  if (NT % cpr == 0) {
    hipLaunchKernelGGL(bn_apply_kernel<true>, dim3(grid_for(M, (NT / cpr) * 4, 8192)), dim3(NT), 0, s, y, scale, shift, r,
                       rscale, rshift, relu, out, M, C, mask);
  } else {
    hipLaunchKernelGGL(bn_apply_kernel<false>, dim3(grid_for(M * cpr, NT * 4, 8192)), dim3(NT), 0, s, y, scale, shift,
                       r, rscale, rshift, relu, out, M, C, mask);
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
// Eligibility of the finalize-in-apply kernels: 64-channel slices, <= FIN_SHARDS shards.
int tfk_bn_fin_ok(int C, int shards) { return (C % 64 == 0 && shards >= 1 && shards <= FIN_SHARDS) ? 1 : 0; }

int tfk_bn_apply_fin(const bf16* y, const BnFin* f, const bf16* r, const BnFin* f2, int relu, bf16* out, long long M, int C,
                     unsigned char* mask, hipStream_t s) {
  if (!tfk_bn_fin_ok(C, f->stats ? f->shards : 1) || (f2 && f2->stats && f2->shards > FIN_SHARDS)) return -2;
  long long rpb;
  const dim3 grid = fin_grid(M, C, &rpb);
  BnFin none{};
  hipLaunchKernelGGL(bn_apply_fin_kernel, grid, dim3(NT), 0, s, y, *f, r, f2 ? *f2 : none, f2 ? 1 : 0, relu, out, M, C,
                     mask, rpb);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int tfk_bn_bwd_apply_fin(const bf16* da, const bf16* y, const float* sums, int shards, const BnBwdFin* f, const bf16* y2,
                         const BnBwdFin* f2, bf16* dy, bf16* dy2, bf16* dres, long long M, int C, const float* mscale,
                         const float* mshift, const unsigned char* amask, hipStream_t s) {
  if (!tfk_bn_fin_ok(C, shards) || (y2 && !f2)) return -2;
  long long rpb;
  const dim3 grid = fin_grid(M, C, &rpb);
  BnBwdFin none{};
  hipLaunchKernelGGL(bn_bwd_apply_fin_kernel, grid, dim3(NT), 0, s, da, y, sums, shards, *f, y2, f2 ? *f2 : none, dy, dy2,
                     dres, M, C, mscale, mshift, amask, rpb);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int tfk_bn_zero(float* p, long long n, hipStream_t s) {
  hipLaunchKernelGGL(bn_zero_kernel, dim3((unsigned)((n + NT * 4 - 1) / (NT * 4))), dim3(NT), 0, s, p, n);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int tfk_bn_bwd_reduce(const bf16* da, const bf16* a, const bf16* y, const float* mean, const float* invstd, const bf16* y2,
                      const float* mean2, const float* invstd2, long long M, int C, float* sums, int shards,
                      const float* mscale, const float* mshift, const unsigned char* amask, hipStream_t s) {
  int cpr = C / 8, rows_par = NT / cpr > 0 ? NT / cpr : 1;
  hipLaunchKernelGGL(bn_bwd_reduce_kernel, dim3(grid_for(M, rows_par * 16, 2048)), dim3(NT), 0, s, da, a, y, mean, invstd,
                     y2, mean2, invstd2, M, C, sums, shards, mscale, mshift, amask);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int tfk_bn_bwd_finalize(float* sums, int shards, int C, float count, const float* gamma, const float* mean,
                        const float* invstd, const float* gamma2, const float* mean2, const float* invstd2,
                        float* dgamma, float* dbeta, float* dgamma2, float* dbeta2, float* coef, float* coef2,
                        hipStream_t s) {
  if (g_fin_skip & 2) return 0;
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 63) / 64), dim3(256), 0, s, sums, shards, C, count, gamma, mean,
                     invstd, gamma2, mean2, invstd2, dgamma, dbeta, dgamma2, dbeta2, coef, coef2);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int tfk_bn_bwd_apply(const bf16* da, const bf16* a, const bf16* y, const float* coef, bf16* dy, const bf16* y2,
                     const float* coef2, bf16* dy2, bf16* dres, long long M, int C, const float* mscale,
                     const float* mshift, const unsigned char* amask, hipStream_t s) {
  const int cpr = C / 8;
  if (NT % cpr == 0) {
    hipLaunchKernelGGL(bn_bwd_apply_kernel<true>, dim3(grid_for(M, (NT / cpr) * 4, 8192)), dim3(NT), 0, s, da, a, y, coef,
                       dy, y2, coef2, dy2, dres, M, C, mscale, mshift, amask);
  } else {
    hipLaunchKernelGGL(bn_bwd_apply_kernel<false>, dim3(grid_for(M * cpr, NT * 4, 8192)), dim3(NT), 0, s, da, a, y,
                       coef, dy, y2, coef2, dy2, dres, M, C, mscale, mshift, amask);
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
}
