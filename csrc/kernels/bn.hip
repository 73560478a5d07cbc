// Training-mode BatchNorm for NHWC bf16 activations [M = N*H*W][C], C % 8 == 0.
//
// Forward statistics are accumulated by the producing conv's GEMM epilogue (gemm.hip, sharded
// f32 atomics), so the forward here is: finalize (shards -> mean/invstd/scale/shift, running
// stats) + one fused apply pass  a = relu(y*scale + shift [+ r | + r*rscale + rshift]).
// The dual-input form fuses a projection shortcut's BN into the residual add of the block.
// Backward: reduce (sum dz, sum dz*xhat[, sum dz*xhat2]) -> finalize (dgamma/dbeta + apply
// coefficients) -> apply (dy[, dy2 | dres]), where dz = da * 1[a > 0].
#include "common.h"

namespace {
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
__global__ void bn_apply_kernel(const bf16* __restrict__ y, const float* __restrict__ scale, const float* __restrict__ shift,
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
__global__ void bn_bwd_apply_kernel(const bf16* __restrict__ da, const bf16* __restrict__ a, const bf16* __restrict__ y,
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
