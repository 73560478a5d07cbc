// Fused optimizers over the executor's FLAT parameter arena (one launch per parameter group,
// no per-tensor multi-tensor-apply lists needed): f32 master weights, f32 grads, f32 slots, and
// the bf16 compute copy refreshed in the same pass. grad_scale may be a device scalar (global-norm
// clipping / loss-scale) so nothing synchronises with the host.
#include "common.h"
#include <cstdlib>

namespace {
constexpr int NT = 256;

__device__ __forceinline__ float gscale_of(float host, const float* dev) { return dev ? host * dev[0] : host; }
// Device hyper-parameters (hipGraph-safe schedules): hp = {lr, bc1, bc2} written on device each
// step by opt_hyper_kernel; a null hp means the host values passed at launch.
__device__ __forceinline__ float hp_or(const float* hp, int i, float host) { return hp ? hp[i] : host; }

__global__ void sgd_kernel(float* __restrict__ w, bf16* __restrict__ wb, const float* __restrict__ g, float* __restrict__ m,
                           long long n, float lr_h, float mu, float wd, int nesterov, float gs_host, const float* gs_dev,
                           const float* hp) {
  const float gs = gscale_of(gs_host, gs_dev);
  const float lr = hp_or(hp, 0, lr_h);
  for (long long i = ((long long)blockIdx.x * NT + threadIdx.x) * 4; i < n; i += (long long)gridDim.x * NT * 4) {
    if (i + 3 < n) {
      f32x4 wv = *(f32x4*)(w + i), gv = *(const f32x4*)(g + i), mv = *(f32x4*)(m + i);
      f32x4 d = gv * gs + wd * wv;
      mv = mu * mv + d;
      f32x4 step = nesterov ? d + mu * mv : mv;
      wv = wv - lr * step;
      *(f32x4*)(w + i) = wv;
      *(f32x4*)(m + i) = mv;
      if (wb) {
        bf16x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = f2bf(wv[e]);
        *(bf16x4*)(wb + i) = o;
      }
    } else {
      for (long long j = i; j < n; ++j) {
        float d = g[j] * gs + wd * w[j];
        m[j] = mu * m[j] + d;
        w[j] -= lr * (nesterov ? d + mu * m[j] : m[j]);
        if (wb) wb[j] = f2bf(w[j]);
      }
    }
  }
}

__global__ void adamw_kernel(float* __restrict__ w, bf16* __restrict__ wb, const float* __restrict__ g, float* __restrict__ m,
                             float* __restrict__ v, long long n, float lr_h, float b1, float b2, float eps, float wd,
                             float bc1, float bc2, float gs_host, const float* gs_dev, const float* hp) {
  const float gs = gscale_of(gs_host, gs_dev);
  const float lr = hp_or(hp, 0, lr_h);
  const float ibc1 = 1.f / hp_or(hp, 1, bc1), ibc2 = 1.f / hp_or(hp, 2, bc2);
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) {
    float gr = g[i] * gs;
    float mm = b1 * m[i] + (1.f - b1) * gr;
    float vv = b2 * v[i] + (1.f - b2) * gr * gr;
    m[i] = mm;
    v[i] = vv;
    float ww = w[i];
    ww -= lr * ((mm * ibc1) / (sqrtf(vv * ibc2) + eps) + wd * ww);
    w[i] = ww;
    if (wb) wb[i] = f2bf(ww);
  }
}

// Vector AdamW: each thread updates TWO float4s per iteration with every load of both issued
// before any math (8 x 16-B streams in flight per thread; the update is HBM-bound, ~30 B/param),
// nontemporal (streaming) loads and stores -- the optimizer touches each byte once per step, so it
// should not evict the GEMM working set from L2 -- and a resident grid (8 blocks per CU). Same
// arithmetic as the scalar adamw_kernel, bit for bit. Needs w, g, m, v 16-B and wb 8-B aligned.
__device__ __forceinline__ float4 ntl(const float4* p) {
  float4 r;
  r.x = __builtin_nontemporal_load(&p->x); r.y = __builtin_nontemporal_load(&p->y);
  r.z = __builtin_nontemporal_load(&p->z); r.w = __builtin_nontemporal_load(&p->w);
  return r;
}
__device__ __forceinline__ void nts(float4* p, float4 v) {
  __builtin_nontemporal_store(v.x, &p->x); __builtin_nontemporal_store(v.y, &p->y);
  __builtin_nontemporal_store(v.z, &p->z); __builtin_nontemporal_store(v.w, &p->w);
}
__global__ __launch_bounds__(NT) void adamw4x2_kernel(float* __restrict__ w, bf16* __restrict__ wb,
                                                      const float* __restrict__ g, float* __restrict__ m,
                                                      float* __restrict__ v, long long n4, float lr_h, float b1,
                                                      float b2, float eps, float wd, float bc1, float bc2,
                                                      float gs_host, const float* gs_dev, const float* hp) {
  const float gs = gscale_of(gs_host, gs_dev);
  const float lr = hp_or(hp, 0, lr_h);
  const float ibc1 = 1.f / hp_or(hp, 1, bc1), ibc2 = 1.f / hp_or(hp, 2, bc2);
  const long long stride = (long long)gridDim.x * NT;
  for (long long i0 = (long long)blockIdx.x * NT + threadIdx.x; i0 < n4; i0 += 2 * stride) {
    const long long i1 = i0 + stride;
    const bool two = i1 < n4;
    float4 gr[2], mm[2], vv[2], ww[2];
    gr[0] = ntl((const float4*)g + i0); mm[0] = ntl((const float4*)m + i0);
    vv[0] = ntl((const float4*)v + i0); ww[0] = ntl((const float4*)w + i0);
    if (two) {
      gr[1] = ntl((const float4*)g + i1); mm[1] = ntl((const float4*)m + i1);
      vv[1] = ntl((const float4*)v + i1); ww[1] = ntl((const float4*)w + i1);
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      if (k == 1 && !two) break;
      float a[4] = {gr[k].x, gr[k].y, gr[k].z, gr[k].w}, b[4] = {mm[k].x, mm[k].y, mm[k].z, mm[k].w};
      float c[4] = {vv[k].x, vv[k].y, vv[k].z, vv[k].w}, d[4] = {ww[k].x, ww[k].y, ww[k].z, ww[k].w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float gg = a[e] * gs;
        b[e] = b1 * b[e] + (1.f - b1) * gg;
        c[e] = b2 * c[e] + (1.f - b2) * gg * gg;
        d[e] -= lr * ((b[e] * ibc1) / (sqrtf(c[e] * ibc2) + eps) + wd * d[e]);
      }
      const long long i = k ? i1 : i0;
      nts((float4*)m + i, make_float4(b[0], b[1], b[2], b[3]));
      nts((float4*)v + i, make_float4(c[0], c[1], c[2], c[3]));
      nts((float4*)w + i, make_float4(d[0], d[1], d[2], d[3]));
      if (wb) {
        bf16 o[4] = {f2bf(d[0]), f2bf(d[1]), f2bf(d[2]), f2bf(d[3])};
        *(uint2*)(wb + 4 * i) = *(const uint2*)o;
      }
    }
  }
}

// LAMB stage 1: u = adam_dir + wd*w written into `u`; per-segment ||w||^2, ||u||^2 via atomics.
// seg_of_chunk: segment id of each 4096-element chunk (host-built; chunks never straddle segments).
__global__ void lamb_stage1_kernel(const float* __restrict__ w, const float* __restrict__ g, float* __restrict__ m,
                                   float* __restrict__ v, float* __restrict__ u, const long long* __restrict__ chunk_start,
                                   const int* __restrict__ chunk_len, const int* __restrict__ chunk_seg, int nchunks,
                                   float b1, float b2, float eps, float wd, float bc1_h, float bc2_h,
                                   float* __restrict__ seg_norms, float gs_host, const float* gs_dev, const float* hp) {
  __shared__ float red[NT / 64];
  const float gs = gscale_of(gs_host, gs_dev);
  const float bc1 = hp_or(hp, 1, bc1_h), bc2 = hp_or(hp, 2, bc2_h);
  for (int c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const long long s0 = chunk_start[c];
    const int len = chunk_len[c];
    float wsq = 0.f, usq = 0.f;
    for (int j = threadIdx.x; j < len; j += NT) {
      long long i = s0 + j;
      float gr = g[i] * gs;
      float mm = b1 * m[i] + (1.f - b1) * gr;
      float vv = b2 * v[i] + (1.f - b2) * gr * gr;
      m[i] = mm;
      v[i] = vv;
      float uu = (mm / bc1) / (sqrtf(vv / bc2) + eps) + wd * w[i];
      u[i] = uu;
      wsq += w[i] * w[i];
      usq += uu * uu;
    }
    wsq = block_sum<NT>(wsq, red);
    usq = block_sum<NT>(usq, red);
    if (threadIdx.x == 0) {
      atomicAdd(seg_norms + 2 * chunk_seg[c], wsq);
      atomicAdd(seg_norms + 2 * chunk_seg[c] + 1, usq);
    }
  }
}

__global__ void lamb_stage2_kernel(float* __restrict__ w, bf16* __restrict__ wb, const float* __restrict__ u,
                                   const long long* __restrict__ chunk_start, const int* __restrict__ chunk_len,
                                   const int* __restrict__ chunk_seg, int nchunks, const float* __restrict__ seg_norms,
                                   float lr_h, const float* hp) {
  const float lr = hp_or(hp, 0, lr_h);
  for (int c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const int sg = chunk_seg[c];
    const float wn = sqrtf(seg_norms[2 * sg]), un = sqrtf(seg_norms[2 * sg + 1]);
    const float ratio = (wn > 0.f && un > 0.f) ? wn / un : 1.f;
    const long long s0 = chunk_start[c];
    const int len = chunk_len[c];
    for (int j = threadIdx.x; j < len; j += NT) {
      long long i = s0 + j;
      float ww = w[i] - lr * ratio * u[i];
      w[i] = ww;
      if (wb) wb[i] = f2bf(ww);
    }
  }
}

// One step of the device schedule: step += 1 (the count of updates applied, TF global_step
// semantics); lr = table[min(step - 1 + lr_offset, T - 1)]; Adam bias corrections 1 - b^step.
__global__ void opt_hyper_kernel(int* step, const float* lr_table, int T, int lr_offset, float b1, float b2, float* hp) {
  const int s = step[0] + 1;
  step[0] = s;
  const int i = min(max(s - 1 + lr_offset, 0), T - 1);
  hp[0] = lr_table[i];
  hp[1] = 1.f - powf(b1, (float)s);
  hp[2] = 1.f - powf(b2, (float)s);
}

// out[0] += sum(x^2) (global grad norm)
__global__ void sumsq_kernel(const float* __restrict__ x, long long n, float* __restrict__ out) {
  __shared__ float red[NT / 64];
  float s = 0.f;
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) s += x[i] * x[i];
  s = block_sum<NT>(s, red);
  if (threadIdx.x == 0) atomicAdd(out, s);
}

// clip coefficient from sumsq: out = min(1, max_norm / (sqrt(ss) + 1e-6)); also stores the norm.
__global__ void clip_coef_kernel(const float* ss, float max_norm, float* coef, float* norm) {
  float nn = sqrtf(ss[0]);
  if (norm) norm[0] = nn;
  coef[0] = max_norm > 0.f ? fminf(1.f, max_norm / (nn + 1e-6f)) : 1.f;
}

int grid_for(long long work, int cap = 4096) {
  long long g = (work + NT - 1) / NT;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}
}  // namespace

extern "C" {
int tfk_sgd(float* w, bf16* wb, const float* g, float* m, long long n, float lr, float mu, float wd, int nesterov,
            float gs, const float* gs_dev, const float* hp, hipStream_t s) {
  hipLaunchKernelGGL(sgd_kernel, dim3(grid_for(n / 4 + 1)), dim3(NT), 0, s, w, wb, g, m, n, lr, mu, wd, nesterov, gs, gs_dev,
                     hp);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int tfk_adamw(float* w, bf16* wb, const float* g, float* m, float* v, long long n, float lr, float b1, float b2, float eps,
              float wd, float bc1, float bc2, float gs, const float* gs_dev, const float* hp, hipStream_t s) {
  const bool vec = (((uintptr_t)w | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) == 0 && (((uintptr_t)wb) & 7) == 0;
  if (vec && n >= 4) {
    const long long n4 = n / 4, done = n4 * 4;
    hipLaunchKernelGGL(adamw4x2_kernel, dim3(grid_for(n4, 2048)), dim3(NT), 0, s, w, wb, g, m, v, n4, lr, b1, b2, eps,
                       wd, bc1, bc2, gs, gs_dev, hp);
    if (done < n)
      hipLaunchKernelGGL(adamw_kernel, dim3(1), dim3(NT), 0, s, w + done, wb ? wb + done : nullptr, g + done, m + done,
                         v + done, n - done, lr, b1, b2, eps, wd, bc1, bc2, gs, gs_dev, hp);
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
  hipLaunchKernelGGL(adamw_kernel, dim3(grid_for(n)), dim3(NT), 0, s, w, wb, g, m, v, n, lr, b1, b2, eps, wd, bc1, bc2, gs,
                     gs_dev, hp);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int tfk_lamb(float* w, bf16* wb, const float* g, float* m, float* v, float* u, const long long* cstart, const int* clen,
             const int* cseg, int nchunks, float* seg_norms, float lr, float b1, float b2, float eps, float wd, float bc1,
             float bc2, float gs, const float* gs_dev, const float* hp, hipStream_t s) {
  int grid = nchunks < 4096 ? nchunks : 4096;
  if (grid < 1) return 0;
  hipLaunchKernelGGL(lamb_stage1_kernel, dim3(grid), dim3(NT), 0, s, w, g, m, v, u, cstart, clen, cseg, nchunks, b1, b2, eps,
                     wd, bc1, bc2, seg_norms, gs, gs_dev, hp);
  hipLaunchKernelGGL(lamb_stage2_kernel, dim3(grid), dim3(NT), 0, s, w, wb, u, cstart, clen, cseg, nchunks, seg_norms, lr,
                     hp);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int tfk_opt_hyper(int* step, const float* lr_table, int T, int lr_offset, float b1, float b2, float* hp, hipStream_t s) {
  hipLaunchKernelGGL(opt_hyper_kernel, dim3(1), dim3(1), 0, s, step, lr_table, T, lr_offset, b1, b2, hp);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int tfk_sumsq(const float* x, long long n, float* out, hipStream_t s) {
  hipLaunchKernelGGL(sumsq_kernel, dim3(grid_for(n, 2048)), dim3(NT), 0, s, x, n, out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int tfk_clip_coef(const float* ss, float max_norm, float* coef, float* norm, hipStream_t s) {
  hipLaunchKernelGGL(clip_coef_kernel, dim3(1), dim3(1), 0, s, ss, max_norm, coef, norm);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
}
