// Fused softmax cross-entropy forward+backward (label smoothing, ignore_index) for gfx950.
// One 256-thread block per row; logits bf16 [B][V]; writes per-row loss (f32) and
// dlogits = scale * (softmax - target) in bf16 in the same kernel. Rows up to 40960 logits are held in
// registers (xent_reg_kernel: one HBM read + one write); longer rows stream (xent_kernel).
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

// Register-resident variant for vocab rows up to CH*NT*8 logits (V=33708 Transformer-big, 30522
// BERT): the row is read from HBM once into VGPRs (CH 16-B chunks per lane) and the max/argmax,
// sum-exp and gradient passes run from registers -- one read + one write of the row instead of
// three reads + one write. Same arithmetic and tie-breaking as xent_kernel.
template <int CH>
__global__ __launch_bounds__(NT) void xent_reg_kernel(const bf16* __restrict__ logits, const int* __restrict__ labels,
                                                      int V, long long ld, float smoothing, int ignore_index,
                                                      float scale, float* __restrict__ loss,
                                                      bf16* __restrict__ dlogits, float* __restrict__ correct) {
  __shared__ float red[NT / 64];
  __shared__ int redi[NT / 64];
  const int row = blockIdx.x;
  const bf16* x = logits + (long long)row * ld;
  const int label = labels[row];
  const int nch = (V + 7) >> 3;  // the last chunk may run into the row padding (ld % 8 == 0, ld >= V)
  bf16x8 v[CH];
  float mx = -INFINITY;
  int amax = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int i = threadIdx.x + c * NT;
    if (i < nch) {
      v[c] = *(const bf16x8*)(x + i * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float f = bf2f(v[c][e]);
        if (i * 8 + e < V && f > mx) { mx = f; amax = i * 8 + e; }
      }
    }
  }
  const float rmax = block_max<NT>(mx, red);
  int cand = (mx == rmax) ? amax : 0x7fffffff;
  for (int o = 32; o > 0; o >>= 1) cand = min(cand, __shfl_xor(cand, o, 64));
  __syncthreads();
  if ((threadIdx.x & 63) == 0) redi[threadIdx.x >> 6] = cand;
  __syncthreads();
  int best = redi[0];
  for (int i = 1; i < NT / 64; ++i) best = min(best, redi[i]);
  float se = 0.f, sx = 0.f;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int i = threadIdx.x + c * NT;
    if (i < nch) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        if (i * 8 + e < V) { const float f = bf2f(v[c][e]); se += __expf(f - rmax); sx += f; }
      }
    }
  }
  se = block_sum<NT>(se, red);
  sx = block_sum<NT>(sx, red);
  const float lse = rmax + __logf(se);
  const bool valid = label != ignore_index && label >= 0 && label < V;
  if (threadIdx.x == 0) {
    float l = 0.f;
    if (valid) {
      const float xl = bf2f(x[label]);
      l = (1.f - smoothing) * (lse - xl) + smoothing * (lse - sx / V);
    }
    loss[row] = l;
    if (correct) correct[row] = (valid && best == label) ? 1.f : 0.f;
  }
  if (!dlogits) return;
  bf16* d = dlogits + (long long)row * ld;
  const float inv_se = 1.f / se, off = smoothing / V, sc = valid ? scale : 0.f;
  const int nw = (int)(ld >> 3);  // every chunk of the padded row is written (padding -> 0)
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int i = threadIdx.x + c * NT;
    if (i >= nch && i < nw) *(bf16x8*)(d + i * 8) = bf16x8{};
    if (i < nch) {
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int j = i * 8 + e;
        const float p = __expf(bf2f(v[c][e]) - rmax) * inv_se;
        const float t = off + (j == label ? 1.f - smoothing : 0.f);
        o[e] = f2bf(j < V ? sc * (p - t) : 0.f);  // padding columns get a zero gradient
      }
      *(bf16x8*)(d + i * 8) = o;
    }
  }
}
constexpr int XENT_REG_CH = 20;  // V <= 40960
// TFK_XENT_REG=0 selects the three-pass streaming kernel (A/B measurements, tests).
static bool xent_reg_on() {
  static const int on = [] { const char* e = getenv("TFK_XENT_REG"); return (e && e[0] == '0') ? 0 : 1; }();
  return on != 0;
}
}  // namespace

// 1 when the launcher takes the register kernel, which writes every column of the padded dlogits row
// (callers can then skip zero-filling the padding).
extern "C" int tfk_xent_full_row(int V, long long ld) {
  return (ld % 8 == 0 && ld >= V && ld / 8 <= XENT_REG_CH * NT && xent_reg_on()) ? 1 : 0;
}

extern "C" int tfk_softmax_xent(const bf16* logits, const int* labels, int B, int V, long long ld, float smoothing,
                                int ignore_index, float scale, float* loss, bf16* dlogits, float* correct, hipStream_t s) {
  if (tfk_xent_full_row(V, ld)) {
    hipLaunchKernelGGL(xent_reg_kernel<XENT_REG_CH>, dim3(B), dim3(NT), 0, s, logits, labels, V, ld, smoothing,
                       ignore_index, scale, loss, dlogits, correct);
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
  hipLaunchKernelGGL(xent_kernel, dim3(B), dim3(NT), 0, s, logits, labels, V, ld, smoothing, ignore_index, scale, loss,
                     dlogits, correct);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
