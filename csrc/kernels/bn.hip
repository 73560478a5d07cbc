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

// ---------------------------------------------------------------- forward
// stats: [shards][2][C] (sum, sumsq), zeroed again after reading so the next conv can accumulate.
__global__ void bn_finalize_kernel(float* stats, int shards, int C, float count, const float* __restrict__ gamma,
                                   const float* __restrict__ beta, float eps, float momentum, float* __restrict__ run_mean,
                                   float* __restrict__ run_var, float* __restrict__ mean_out, float* __restrict__ invstd_out,
                                   float* __restrict__ scale_out, float* __restrict__ shift_out) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float s = 0.f, q = 0.f;
#pragma unroll 8
  for (int i = 0; i < shards; ++i) {
    s += stats[(long long)i * 2 * C + c];
    q += stats[(long long)i * 2 * C + C + c];
  }
#pragma unroll 8
  for (int i = 0; i < shards; ++i) {
    stats[(long long)i * 2 * C + c] = 0.f;
    stats[(long long)i * 2 * C + C + c] = 0.f;
  }
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

__global__ void bn_apply_kernel(const bf16* __restrict__ y, const float* __restrict__ scale, const float* __restrict__ shift,
                                const bf16* __restrict__ r, const float* __restrict__ rscale, const float* __restrict__ rshift,
                                int relu, bf16* __restrict__ out, long long nchunks, int C) {
  const int cpr = C >> 3;
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < nchunks; i += (long long)gridDim.x * NT) {
    const int c0 = (int)(i % cpr) * 8;
    bf16x8 v = *(const bf16x8*)(y + i * 8);
    f32x4 s0 = *(const f32x4*)(scale + c0), s1 = *(const f32x4*)(scale + c0 + 4);
    f32x4 b0 = *(const f32x4*)(shift + c0), b1 = *(const f32x4*)(shift + c0 + 4);
    float o[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) { o[e] = bf2f(v[e]) * s0[e] + b0[e]; o[e + 4] = bf2f(v[e + 4]) * s1[e] + b1[e]; }
    if (r) {
      bf16x8 rv = *(const bf16x8*)(r + i * 8);
      if (rscale) {
        f32x4 rs0 = *(const f32x4*)(rscale + c0), rs1 = *(const f32x4*)(rscale + c0 + 4);
        f32x4 rb0 = *(const f32x4*)(rshift + c0), rb1 = *(const f32x4*)(rshift + c0 + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) { o[e] += bf2f(rv[e]) * rs0[e] + rb0[e]; o[e + 4] += bf2f(rv[e + 4]) * rs1[e] + rb1[e]; }
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] += bf2f(rv[e]);
      }
    }
    bf16x8 w;
#pragma unroll
    for (int e = 0; e < 8; ++e) w[e] = f2bf(relu ? fmaxf(o[e], 0.f) : o[e]);
    *(bf16x8*)(out + i * 8) = w;
  }
}

// ---------------------------------------------------------------- backward
// sums: [shards][3][C]: sum dz, sum dz*xhat, sum dz*xhat2
__global__ void bn_bwd_reduce_kernel(const bf16* __restrict__ da, const bf16* __restrict__ a, const bf16* __restrict__ y,
                                     const float* __restrict__ mean, const float* __restrict__ invstd,
                                     const bf16* __restrict__ y2, const float* __restrict__ mean2,
                                     const float* __restrict__ invstd2, long long M, int C, float* __restrict__ sums,
                                     int shards, const float* __restrict__ mscale, const float* __restrict__ mshift) {
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
      bf16x8 y2v;
      if (y2) y2v = *(const bf16x8*)(y2 + off);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float dz = bf2f(g[e]);
        if (a && !(bf2f(av[e]) > 0.f)) dz = 0.f;
        if (!a && mscale && !(bf2f(yv[e]) * msc[e] + msh[e] > 0.f)) dz = 0.f;
        s0[e] += dz;
        s1[e] += dz * (bf2f(yv[e]) - mu[e]) * is[e];
        if (y2) s2[e] += dz * (bf2f(y2v[e]) - mu2[e]) * is2[e];
      }
    }
  }
  __shared__ float red[NT * 8];
  float* st = sums + (long long)(blockIdx.x % shards) * 3 * C;
  const int npass = y2 ? 3 : 2;
  for (int pass = 0; pass < npass; ++pass) {
    float* src = pass == 0 ? s0 : (pass == 1 ? s1 : s2);
    __syncthreads();
#pragma unroll
    for (int e = 0; e < 8; ++e) red[t * 8 + e] = src[e];
    __syncthreads();
    if (rsub == 0) {
      for (int rr = 1; rr < rows_par; ++rr)
#pragma unroll
        for (int e = 0; e < 8; ++e) src[e] += red[(rr * cpr + cchunk) * 8 + e];
#pragma unroll
      for (int e = 0; e < 8; ++e) atomicAdd(st + pass * C + c0 + e, src[e]);
    }
  }
}

// Reduce shards; write dgamma/dbeta (+= if accumulate) and per-channel apply coefficients
// coef: [k1, k2, k3][C] with dy = k1*(dz - k2 - xhat*k3); coef2 same for the second BN.
__global__ void bn_bwd_finalize_kernel(float* sums, int shards, int C, float count,
                                       const float* __restrict__ gamma, const float* __restrict__ invstd,
                                       const float* __restrict__ gamma2, const float* __restrict__ invstd2,
                                       float* __restrict__ dgamma, float* __restrict__ dbeta, float* __restrict__ dgamma2,
                                       float* __restrict__ dbeta2, float* __restrict__ coef, float* __restrict__ coef2) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f;
#pragma unroll 8
  for (int i = 0; i < shards; ++i) {
    const float* p = sums + (long long)i * 3 * C;
    s0 += p[c]; s1 += p[C + c]; s2 += p[2 * C + c];
  }
#pragma unroll 8
  for (int i = 0; i < shards; ++i) {
    float* p = sums + (long long)i * 3 * C;
    p[c] = 0.f; p[C + c] = 0.f; p[2 * C + c] = 0.f;
  }
  dgamma[c] = s1;
  dbeta[c] = s0;
  coef[c] = gamma[c] * invstd[c];
  coef[C + c] = s0 / count;
  coef[2 * C + c] = s1 / count;
  if (coef2) {
    dgamma2[c] = s2;
    dbeta2[c] = s0;
    coef2[c] = gamma2[c] * invstd2[c];
    coef2[C + c] = s0 / count;
    coef2[2 * C + c] = s2 / count;
  }
}

// dy = k1*(dz - k2 - xhat*k3); optional dy2 (projection-shortcut BN) or dres = dz (identity shortcut).
__global__ void bn_bwd_apply_kernel(const bf16* __restrict__ da, const bf16* __restrict__ a, const bf16* __restrict__ y,
                                    const float* __restrict__ mean, const float* __restrict__ invstd,
                                    const float* __restrict__ coef, bf16* __restrict__ dy, const bf16* __restrict__ y2,
                                    const float* __restrict__ mean2, const float* __restrict__ invstd2,
                                    const float* __restrict__ coef2, bf16* __restrict__ dy2, bf16* __restrict__ dres,
                                    long long nchunks, int C, const float* __restrict__ mscale,
                                    const float* __restrict__ mshift) {
  const int cpr = C >> 3;
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < nchunks; i += (long long)gridDim.x * NT) {
    const int c0 = (int)(i % cpr) * 8;
    bf16x8 g = *(const bf16x8*)(da + i * 8);
    bf16x8 yv = *(const bf16x8*)(y + i * 8);
    bf16x8 av;
    if (a) av = *(const bf16x8*)(a + i * 8);
    float dz[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      dz[e] = bf2f(g[e]);
      if (a && !(bf2f(av[e]) > 0.f)) dz[e] = 0.f;
      if (!a && mscale && !(bf2f(yv[e]) * mscale[c0 + e] + mshift[c0 + e] > 0.f)) dz[e] = 0.f;
    }
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = c0 + e;
      float xh = (bf2f(yv[e]) - mean[c]) * invstd[c];
      o[e] = f2bf(coef[c] * (dz[e] - coef[C + c] - xh * coef[2 * C + c]));
    }
    *(bf16x8*)(dy + i * 8) = o;
    if (y2) {
      bf16x8 y2v = *(const bf16x8*)(y2 + i * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = c0 + e;
        float xh = (bf2f(y2v[e]) - mean2[c]) * invstd2[c];
        o[e] = f2bf(coef2[c] * (dz[e] - coef2[C + c] - xh * coef2[2 * C + c]));
      }
      *(bf16x8*)(dy2 + i * 8) = o;
    }
    if (dres) {
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = f2bf(dz[e]);
      *(bf16x8*)(dres + i * 8) = o;
    }
  }
}

int grid_for(long long work, int per_block, int cap = 4096) {
  long long g = (work + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}
}  // namespace

extern "C" {
int tfk_bn_finalize(float* stats, int shards, int C, float count, const float* gamma, const float* beta, float eps,
                    float momentum, float* run_mean, float* run_var, float* mean, float* invstd, float* scale,
                    float* shift, hipStream_t s) {
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + 63) / 64), dim3(64), 0, s, stats, shards, C, count, gamma, beta, eps,
                     momentum, run_mean, run_var, mean, invstd, scale, shift);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int tfk_bn_stats(const bf16* y, long long M, int C, float* stats, int shards, hipStream_t s) {
  int cpr = C / 8, rows_par = NT / cpr > 0 ? NT / cpr : 1;
  hipLaunchKernelGGL(bn_stats_kernel, dim3(grid_for(M, rows_par * 16, 2048)), dim3(NT), 0, s, y, M, C, stats, shards);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int tfk_bn_apply(const bf16* y, const float* scale, const float* shift, const bf16* r, const float* rscale,
                 const float* rshift, int relu, bf16* out, long long M, int C, hipStream_t s) {
  long long nch = M * C / 8;
  hipLaunchKernelGGL(bn_apply_kernel, dim3(grid_for(nch, NT * 4, 8192)), dim3(NT), 0, s, y, scale, shift, r, rscale, rshift,
                     relu, out, nch, C);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int tfk_bn_bwd_reduce(const bf16* da, const bf16* a, const bf16* y, const float* mean, const float* invstd, const bf16* y2,
                      const float* mean2, const float* invstd2, long long M, int C, float* sums, int shards,
                      const float* mscale, const float* mshift, hipStream_t s) {
  int cpr = C / 8, rows_par = NT / cpr > 0 ? NT / cpr : 1;
  hipLaunchKernelGGL(bn_bwd_reduce_kernel, dim3(grid_for(M, rows_par * 16, 2048)), dim3(NT), 0, s, da, a, y, mean, invstd,
                     y2, mean2, invstd2, M, C, sums, shards, mscale, mshift);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int tfk_bn_bwd_finalize(float* sums, int shards, int C, float count, const float* gamma, const float* invstd,
                        const float* gamma2, const float* invstd2, float* dgamma, float* dbeta, float* dgamma2,
                        float* dbeta2, float* coef, float* coef2, hipStream_t s) {
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 63) / 64), dim3(64), 0, s, sums, shards, C, count, gamma, invstd,
                     gamma2, invstd2, dgamma, dbeta, dgamma2, dbeta2, coef, coef2);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int tfk_bn_bwd_apply(const bf16* da, const bf16* a, const bf16* y, const float* mean, const float* invstd,
                     const float* coef, bf16* dy, const bf16* y2, const float* mean2, const float* invstd2,
                     const float* coef2, bf16* dy2, bf16* dres, long long M, int C, const float* mscale,
                     const float* mshift, hipStream_t s) {
  long long nch = M * C / 8;
  hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(grid_for(nch, NT * 4, 8192)), dim3(NT), 0, s, da, a, y, mean, invstd, coef,
                     dy, y2, mean2, invstd2, coef2, dy2, dres, nch, C, mscale, mshift);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
}
