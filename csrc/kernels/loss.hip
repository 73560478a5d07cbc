// Fused softmax cross-entropy forward+backward (label smoothing, ignore_index) for gfx950.
// One 256-thread block per row; logits bf16 [B][V]; writes per-row loss (f32) and
// dlogits = scale * (softmax - target) in bf16 in the same pass (online max/sum, two sweeps).
#include "common.h"

namespace {
constexpr int NT = 256;

__global__ void xent_kernel(const bf16* __restrict__ logits, const int* __restrict__ labels, int V, long long ld,
                            float smoothing, int ignore_index, float scale, float* __restrict__ loss,
                            bf16* __restrict__ dlogits, float* __restrict__ correct) {
  __shared__ float red[NT / 64];
  const int row = blockIdx.x;
  const bf16* x = logits + (long long)row * ld;
  const int label = labels[row];
  const bool vec = (V % 8 == 0) && (ld % 8 == 0);
  // pass 1: max and argmax
  float mx = -INFINITY;
  int amax = 0;
  if (vec) {
    for (int i = threadIdx.x; i < V / 8; i += NT) {
      bf16x8 v = *(const bf16x8*)(x + i * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) { float f = bf2f(v[e]); if (f > mx) { mx = f; amax = i * 8 + e; } }
    }
  } else {
    for (int i = threadIdx.x; i < V; i += NT) { float f = bf2f(x[i]); if (f > mx) { mx = f; amax = i; } }
  }
  const float rmax = block_max<NT>(mx, red);
  // argmax: smallest index achieving the max
  int cand = (mx == rmax) ? amax : 0x7fffffff;
  for (int o = 32; o > 0; o >>= 1) cand = min(cand, __shfl_xor(cand, o, 64));
  __shared__ int redi[NT / 64];
  __syncthreads();
  if ((threadIdx.x & 63) == 0) redi[threadIdx.x >> 6] = cand;
  __syncthreads();
  int best = redi[0];
  for (int i = 1; i < NT / 64; ++i) best = min(best, redi[i]);
  // pass 2: sum exp and sum logits (for smoothing)
  float se = 0.f, sx = 0.f;
  if (vec) {
    for (int i = threadIdx.x; i < V / 8; i += NT) {
      bf16x8 v = *(const bf16x8*)(x + i * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) { float f = bf2f(v[e]); se += __expf(f - rmax); sx += f; }
    }
  } else {
    for (int i = threadIdx.x; i < V; i += NT) { float f = bf2f(x[i]); se += __expf(f - rmax); sx += f; }
  }
  se = block_sum<NT>(se, red);
  sx = block_sum<NT>(sx, red);
  const float lse = rmax + __logf(se);
  const bool valid = label != ignore_index && label >= 0 && label < V;
  if (threadIdx.x == 0) {
    float l = 0.f;
    if (valid) {
      float xl = bf2f(x[label]);
      l = (1.f - smoothing) * (lse - xl) + smoothing * (lse - sx / V);
    }
    loss[row] = l;
    if (correct) correct[row] = (valid && best == label) ? 1.f : 0.f;
  }
  if (!dlogits) return;
  bf16* d = dlogits + (long long)row * ld;
  const float inv_se = 1.f / se, off = smoothing / V, sc = valid ? scale : 0.f;
  if (vec) {
    for (int i = threadIdx.x; i < V / 8; i += NT) {
      bf16x8 v = *(const bf16x8*)(x + i * 8);
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        int j = i * 8 + e;
        float p = __expf(bf2f(v[e]) - rmax) * inv_se;
        float t = off + (j == label ? 1.f - smoothing : 0.f);
        o[e] = f2bf(sc * (p - t));
      }
      *(bf16x8*)(d + i * 8) = o;
    }
  } else {
    for (int j = threadIdx.x; j < V; j += NT) {
      float p = __expf(bf2f(x[j]) - rmax) * inv_se;
      float t = off + (j == label ? 1.f - smoothing : 0.f);
      d[j] = f2bf(sc * (p - t));
    }
  }
}
}  // namespace

extern "C" int tfk_softmax_xent(const bf16* logits, const int* labels, int B, int V, long long ld, float smoothing,
                                int ignore_index, float scale, float* loss, bf16* dlogits, float* correct, hipStream_t s) {
  hipLaunchKernelGGL(xent_kernel, dim3(B), dim3(NT), 0, s, logits, labels, V, ld, smoothing, ignore_index, scale, loss,
                     dlogits, correct);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
