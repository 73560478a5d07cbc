// Small utility kernels for the executor: split-K slab reduction, weight transposes for conv
// dgrad, casts, fills, on-device synthetic data (no H2D in the hot loop), column sums (bias
// grads), elementwise activation/dropout forward+backward.
#include "common.h"

namespace {
constexpr int NT = 256;

int grid_for(long long work, int cap = 8192) {
  long long g = (work + NT - 1) / NT;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

// out[i] = (acc ? out[i] : 0) + alpha * sum_s slabs[s*stride + i]; optional bf16 output instead.
// Two deterministic passes, no atomics. Pass 1: grid (n/256 chunks, G slab groups); a block's 4
// waves take the group's slabs round-robin (16-B loads, 4 elements per lane) and meet in LDS in a
// fixed order; with G == 1 it writes `out` directly, else the group partial goes IN PLACE into the
// group's first slab (only this block reads that chunk of it). Pass 2 (G > 1): partials summed in
// group order. G is chosen so pass 1 has ~1024 blocks: a small weight with hundreds of split-K slabs
// (64x64 1x1 wgrad: 256 slabs x 16K) spreads over the chip instead of 16 blocks walking 256 slabs
// (the previous form: 8-slab groups combined with f32 atomics, 18 us for 16 MB, non-deterministic).
// S <= 8 takes splitk_direct_kernel below instead (one pass, no LDS).
template <bool FINAL>
__device__ __forceinline__ void splitk_store(long long i, long long n, f32x4 a, float* out, bf16* outb,
                                             int accumulate, float alpha) {
  a *= alpha;
  if (i + 3 < n) {
    if (out) {
      if (accumulate) a += *(f32x4*)(out + i);
      *(f32x4*)(out + i) = a;
    } else {
      bf16x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = f2bf(a[e] + (accumulate ? bf2f(outb[i + e]) : 0.f));
      *(bf16x4*)(outb + i) = o;
    }
  } else {
    for (int e = 0; e < 4 && i + e < n; ++e) {
      if (out) out[i + e] = a[e] + (accumulate ? out[i + e] : 0.f);
      else outb[i + e] = f2bf(a[e] + (accumulate ? bf2f(outb[i + e]) : 0.f));
    }
  }
}

__global__ __launch_bounds__(256) void splitk_partial_kernel(float* __restrict__ slabs, int S, int SG, long long stride,
                                                             long long n, float* __restrict__ out, bf16* __restrict__ outb,
                                                             int accumulate, float alpha) {
  __shared__ f32x4 red[3][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long long i = ((long long)blockIdx.x * 64 + lane) * 4;
  const int s0 = blockIdx.y * SG, s1 = min(S, s0 + SG);
  f32x4 a = {0.f, 0.f, 0.f, 0.f};
  if (i + 3 < n) {
#pragma unroll 4
    for (int s = s0 + w; s < s1; s += 4) a += __builtin_nontemporal_load((const f32x4*)(slabs + s * stride + i));
  } else if (i < n) {
    for (int s = s0 + w; s < s1; s += 4)
      for (int e = 0; e < 4 && i + e < n; ++e) a[e] += slabs[s * stride + i + e];
  }
  if (w > 0) red[w - 1][lane] = a;
  __syncthreads();
  if (w != 0 || i >= n) return;
  a += red[0][lane];
  a += red[1][lane];
  a += red[2][lane];
  if (gridDim.y == 1) {
    splitk_store<true>(i, n, a, out, outb, accumulate, alpha);
  } else if (i + 3 < n) {
    *(f32x4*)(slabs + s0 * stride + i) = a;
  } else {
    for (int e = 0; e < 4 && i + e < n; ++e) slabs[s0 * stride + i + e] = a[e];
  }
}

__global__ void splitk_final_kernel(const float* __restrict__ slabs, int G, int SG, long long stride, long long n,
                                    float* __restrict__ out, bf16* __restrict__ outb, int accumulate, float alpha) {
  const long long i = ((long long)blockIdx.x * NT + threadIdx.x) * 4;
  if (i >= n) return;
  f32x4 a = {0.f, 0.f, 0.f, 0.f};
  if (i + 3 < n) {
#pragma unroll 4
    for (int g = 0; g < G; ++g) a += *(const f32x4*)(slabs + (long long)g * SG * stride + i);
  } else {
    for (int g = 0; g < G; ++g)
      for (int e = 0; e < 4 && i + e < n; ++e) a[e] += slabs[(long long)g * SG * stride + i + e];
  }
  splitk_store<true>(i, n, a, out, outb, accumulate, alpha);
}

// Few slabs (S <= 8: the linear weight gradients' split counts, halved on the side streams to 2-4):
// every lane sums its 4-element column of all S slabs itself, U columns 1024 elements apart, with
// all S x U 16-B loads issued before the first add. No LDS, no barrier, no idle waves (the two-pass
// kernel hands each slab to one of 4 waves: at S = 2 half of them idle, and each lane has one load in
// flight). Same summation order as the two-pass kernel's one-group path: a_w = slabs w, w + 4 in
// order, then ((a0 + a1) + a2) + a3 -- bit-identical results.
template <int S, int U>
__global__ __launch_bounds__(256) void splitk_direct_kernel(const float* __restrict__ slabs, long long stride,
                                                            long long n, float* __restrict__ out,
                                                            bf16* __restrict__ outb, int accumulate, float alpha) {
  const long long base = (long long)blockIdx.x * (1024 * U) + threadIdx.x * 4;
  f32x4 v[U][S];
  if ((long long)(blockIdx.x + 1) * (1024 * U) <= n) {  // interior block (uniform): unguarded loads
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int s = 0; s < S; ++s)
        v[u][s] = __builtin_nontemporal_load((const f32x4*)(slabs + s * stride + base + u * 1024));
  } else {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long i = base + u * 1024;
#pragma unroll
      for (int s = 0; s < S; ++s) {
        if (i + 3 < n) {
          v[u][s] = __builtin_nontemporal_load((const f32x4*)(slabs + s * stride + i));
        } else {
          v[u][s] = f32x4{0.f, 0.f, 0.f, 0.f};
          for (int e = 0; e < 4 && i + e < n; ++e) v[u][s][e] = slabs[s * stride + i + e];
        }
      }
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long long i = base + u * 1024;
    if (i >= n) return;
    f32x4 a[4];
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      a[w] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = w; s < S; s += 4) a[w] += v[u][s];
    }
    f32x4 r = a[0];
    r += a[1];
    r += a[2];
    r += a[3];
    splitk_store<true>(i, n, r, out, outb, accumulate, alpha);
  }
}

template <int S>
void splitk_direct_launch(const float* slabs, long long stride, long long n, float* out, bf16* outb, int accumulate,
                          float alpha, int U, hipStream_t s) {
  if (U == 2)
    hipLaunchKernelGGL((splitk_direct_kernel<S, 2>), dim3((unsigned)((n + 2047) / 2048)), dim3(256), 0, s, slabs,
                       stride, n, out, outb, accumulate, alpha);
  else
    hipLaunchKernelGGL((splitk_direct_kernel<S, 1>), dim3((unsigned)((n + 1023) / 1024)), dim3(256), 0, s, slabs,
                       stride, n, out, outb, accumulate, alpha);
}

// 0: two-pass kernel only; 1: S <= 8 direct, one column per lane; 2: direct, two columns per lane
// from 1M elements (A/B knob; TFK_SPLITK_DIRECT=0/1/2, default 2)
int g_splitk_direct = -1;
int splitk_direct_mode() {
  if (g_splitk_direct < 0) {
    const char* e = getenv("TFK_SPLITK_DIRECT");
    g_splitk_direct = (e && e[0] >= '0' && e[0] <= '2') ? e[0] - '0' : 2;
  }
  return g_splitk_direct;
}

// in [A][R][B] -> out [B][R][A] (bf16), 32x32 LDS tiles; grid (ceil(B/32), ceil(A/32), R).
// flip: write middle index R-1-r (a conv weight's (r,s) taps reversed: the stride-1 dgrad as a
// forward conv over dY, ops/gemm.py conv_dgrad).
__global__ void transpose_arb_kernel(const bf16* __restrict__ in, bf16* __restrict__ out, int A, int R, int B,
                                     int flip) {
  __shared__ bf16 tile[32][33];
  const int b0 = blockIdx.x * 32, a0 = blockIdx.y * 32, r = blockIdx.z;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 threads -> 8 rows per pass
  for (int i = ty; i < 32; i += 8) {
    int a = a0 + i, b = b0 + tx;
    tile[i][tx] = (a < A && b < B) ? in[((long long)a * R + r) * B + b] : f2bf(0.f);
  }
  __syncthreads();
  for (int i = ty; i < 32; i += 8) {
    int b = b0 + i, a = a0 + tx;
    if (a < A && b < B) out[((long long)b * R + (flip ? R - 1 - r : r)) * A + a] = tile[tx][i];
  }
}

// 2D transpose [rows][cols] -> [cols][rows] for f32 (weight layout conversions for checkpoints).
__global__ void transpose_f32_kernel(const float* __restrict__ in, float* __restrict__ out, int rows, int cols) {
  __shared__ float tile[32][33];
  const int c0 = blockIdx.x * 32, r0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int i = ty; i < 32; i += 8) {
    int r = r0 + i, c = c0 + tx;
    if (r < rows && c < cols) tile[i][tx] = in[(long long)r * cols + c];
  }
  __syncthreads();
  for (int i = ty; i < 32; i += 8) {
    int c = c0 + i, r = r0 + tx;
    if (r < rows && c < cols) out[(long long)c * rows + r] = tile[tx][i];
  }
}

// Casts (master refresh, MWMS bf16 wire buckets): 4 elements per lane (16-B f32 / 8-B bf16
// accesses) when both pointers are aligned for it; the launcher runs the scalar form otherwise.
__global__ void cast_f32_bf16_kernel(const float* __restrict__ x, bf16* __restrict__ y, long long n) {
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) y[i] = f2bf(x[i]);
}
__global__ void cast_bf16_f32_kernel(const bf16* __restrict__ x, float* __restrict__ y, long long n) {
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) y[i] = bf2f(x[i]);
}
__global__ void cast4_f32_bf16_kernel(const float* __restrict__ x, bf16* __restrict__ y, long long n4) {
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n4; i += (long long)gridDim.x * NT) {
    const f32x4 v = ((const f32x4*)x)[i];
    bf16x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = f2bf(v[e]);
    ((bf16x4*)y)[i] = o;
  }
}
__global__ void cast4_bf16_f32_kernel(const bf16* __restrict__ x, float* __restrict__ y, long long n4) {
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n4; i += (long long)gridDim.x * NT) {
    const bf16x4 v = ((const bf16x4*)x)[i];
    f32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = bf2f(v[e]);
    ((f32x4*)y)[i] = o;
  }
}

// Uniform [lo, hi) bf16 with channel padding: tensor [rows][Cpad], channels >= Creal are zero.
__global__ void synth_uniform_kernel(bf16* __restrict__ y, long long rows, int Creal, int Cpad, float lo, float hi,
                                     unsigned long long seed) {
  const long long n = rows * Cpad;
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) {
    int c = (int)(i % Cpad);
    y[i] = c < Creal ? f2bf(lo + (hi - lo) * u01(hash_u32(seed, i))) : f2bf(0.f);
  }
}
__global__ void synth_normal_f32_kernel(float* __restrict__ y, long long n, float mean, float std, unsigned long long seed) {
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) {
    float u1 = fmaxf(u01(hash_u32(seed, 2 * i)), 1e-7f), u2 = u01(hash_u32(seed, 2 * i + 1));
    y[i] = mean + std * sqrtf(-2.f * __logf(u1)) * __cosf(6.2831853f * u2);
  }
}
__global__ void synth_labels_kernel(int* __restrict__ y, long long n, int classes, unsigned long long seed) {
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT)
    y[i] = (int)(hash_u32(seed, i) % (uint32_t)classes);
}

// Column sums of bf16 [M][N] -> f32 out[N] (bias grads). Block = 64 columns x 4 row-groups.
__global__ void colsum_kernel(const bf16* __restrict__ x, long long M, int N, long long ld, float* __restrict__ out,
                              int accumulate_atomic) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rg = threadIdx.x >> 6;
  float s = 0.f;
  if (c < N)
    for (long long r = (long long)blockIdx.y * 4 + rg; r < M; r += (long long)gridDim.y * 4) s += bf2f(x[r * ld + c]);
  __shared__ float red[4][64];
  red[rg][threadIdx.x & 63] = s;
  __syncthreads();
  if (rg == 0 && c < N) {
    s = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
    atomicAdd(out + c, s);
  }
}

// Vector form (N % 8 == 0, ld % 8 == 0, 16-B aligned rows): each lane sums 8 adjacent columns with
// 16-B loads, so a wave streams 1 KiB per row instead of 128 B; block = 64 lanes x 4 row groups
// covers 512 columns, blockIdx.y splits the rows; partials meet in LDS, one atomic per column.
__global__ void colsum8_kernel(const bf16* __restrict__ x, long long M, int N, long long ld, float* __restrict__ out) {
  const int lane = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int c = (blockIdx.x * 64 + lane) * 8;
  float s[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) s[e] = 0.f;
  if (c < N) {
    // 4 rows' loads in flight per lane (rows past M reload row r; their values are not added): the
    // one-load-per-iteration loop waited one memory latency per row (BERT-base: 14 us per call)
    const long long step = (long long)gridDim.y * 4;
    for (long long r = (long long)blockIdx.y * 4 + rg; r < M; r += 4 * step) {
      bf16x8 v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const long long rk = r + k * step < M ? r + k * step : r;
        v[k] = *(const bf16x8*)(x + rk * ld + c);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (k == 0 || r + k * step < M) {
#pragma unroll
          for (int e = 0; e < 8; ++e) s[e] += bf2f(v[k][e]);
        }
    }
  }
  __shared__ float red[4][512];
#pragma unroll
  for (int e = 0; e < 8; ++e) red[rg][lane * 8 + e] = s[e];
  __syncthreads();
  for (int j = threadIdx.x; j < 512; j += NT) {
    const int col = blockIdx.x * 512 + j;
    if (col < N) atomicAdd(out + col, red[0][j] + red[1][j] + red[2][j] + red[3][j]);
  }
}

// act: 1 relu, 2 gelu(tanh). y = act(x [+ bias[col]]).
__global__ void act_fwd_kernel(const bf16* __restrict__ x, const float* __restrict__ bias, int N, bf16* __restrict__ y,
                               long long n, int act) {
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) {
    float v = bf2f(x[i]) + (bias ? bias[i % N] : 0.f);
    y[i] = f2bf(act_apply(v, act));
  }
}
// dx = dy * act'(x_preact)
__global__ void act_bwd_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ x, bf16* __restrict__ dx, long long n,
                               int act) {
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) {
    float v = bf2f(x[i]), g = bf2f(dy[i]);
    dx[i] = f2bf(g * act_grad(v, act));
  }
}

// Inverted dropout; mask regenerated from (seed, index) in backward -> no mask tensor stored.
__global__ void dropout_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, long long n, float p,
                               unsigned long long salt, const unsigned long long* __restrict__ key) {
  const int thr = drop_thr8(p);
  const float inv = drop_scale8(p);
  const uint32_t s32 = drop_seed32(eff_seed(salt, key));
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) {
    bool k = drop_keep1(s32, (unsigned long long)i, thr);
    y[i] = f2bf(k ? bf2f(x[i]) * inv : 0.f);
  }
}

// Same mask and arithmetic, 8 elements (16 B) per lane: n % 8 == 0, 16-B aligned x / y. The scalar
// form moved one bf16 per lane per iteration (19 us for a 16 MB Transformer-big residual gradient).
__global__ void dropout8_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, long long n8, float p,
                                unsigned long long salt, const unsigned long long* __restrict__ key) {
  const int thr = drop_thr8(p);
  const float inv = drop_scale8(p);
  const uint32_t s32 = drop_seed32(eff_seed(salt, key));
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n8; i += (long long)gridDim.x * NT) {
    const bf16x8 v = *(const bf16x8*)(x + i * 8);
    const unsigned km = drop_keep8(s32, (unsigned long long)i * 8, thr);
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f2bf((km >> e) & 1u ? bf2f(v[e]) * inv : 0.f);
    *(bf16x8*)(y + i * 8) = o;
  }
}

__global__ void add_kernel(const bf16* __restrict__ a, const bf16* __restrict__ b, bf16* __restrict__ y, long long n,
                           float alpha, float beta) {
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT)
    y[i] = f2bf(alpha * bf2f(a[i]) + beta * bf2f(b[i]));
}

// Row gather / scatter-add of BERT's prediction heads (the MLM positions and the [CLS] rows of a
// [B*S][W] activation): GEMM-row r of the head is activation row (r / P) * S + (pos ? pos[r] : 0).
// One 16-B chunk (8 bf16) per lane, rows of W % 8 == 0.
__global__ void gather_rows_kernel(const bf16* __restrict__ src, const int* __restrict__ pos, int P, int S, int W,
                                   long long n_rows, bf16* __restrict__ dst) {
  const int cpr = W / 8;
  const long long total = n_rows * cpr;
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < total; i += (long long)gridDim.x * NT) {
    const long long r = i / cpr;
    const int c = (int)(i - r * cpr);
    const long long b = r / P;
    const long long row = b * S + (pos ? pos[r] : 0);
    *(bf16x8*)(dst + r * W + c * 8) = *(const bf16x8*)(src + row * W + c * 8);
  }
}
// dst[row(r)] += src[r] in f32, rounded to bf16. Block b owns sequence b: its P rows are added one
// after the other (barrier between), so repeated positions inside a sequence accumulate correctly
// and no two blocks ever touch the same destination row (no atomics).
__global__ void scatter_add_rows_kernel(bf16* __restrict__ dst, const bf16* __restrict__ src, const int* __restrict__ pos,
                                        int P, int S, int W) {
  const long long b = blockIdx.x;
  for (int q = 0; q < P; ++q) {
    const long long r = b * P + q;
    const long long row = b * S + (pos ? pos[r] : 0);
    for (int c = threadIdx.x; c < W / 8; c += NT) {
      bf16x8 d = *(const bf16x8*)(dst + row * W + c * 8);
      const bf16x8 v = *(const bf16x8*)(src + r * W + c * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) d[e] = f2bf(bf2f(d[e]) + bf2f(v[e]));
      *(bf16x8*)(dst + row * W + c * 8) = d;
    }
    __syncthreads();  // the next position of this sequence may be the same row
  }
}
}  // namespace

extern "C" {
int tfk_gather_rows(const bf16* src, const int* pos, int P, int S, int W, long long n_rows, bf16* dst, hipStream_t s) {
  if (W % 8 || P < 1 || (((uintptr_t)src | (uintptr_t)dst) & 15)) return -1;
  hipLaunchKernelGGL(gather_rows_kernel, dim3(grid_for(n_rows * (W / 8))), dim3(NT), 0, s, src, pos, P, S, W, n_rows, dst);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int tfk_scatter_add_rows(bf16* dst, const bf16* src, const int* pos, int P, int S, int W, int B, hipStream_t s) {
  if (W % 8 || P < 1 || B < 1 || (((uintptr_t)src | (uintptr_t)dst) & 15)) return -1;
  hipLaunchKernelGGL(scatter_add_rows_kernel, dim3(B), dim3(NT), 0, s, dst, src, pos, P, S, W);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
void tfk_splitk_set_direct(int mode) { g_splitk_direct = mode < 0 || mode > 2 ? 2 : mode; }
int tfk_splitk_reduce(const float* slabs, int S, long long stride, long long n, float* out, bf16* outb, int accumulate,
                      float alpha, hipStream_t s) {
  if (S < 1 || n < 1) return 0;
  const int dmode = splitk_direct_mode();
  if (dmode > 0 && S <= 8) {
    const int U = (dmode == 2 && n >= (1LL << 20)) ? 2 : 1;
    switch (S) {
      case 1: splitk_direct_launch<1>(slabs, stride, n, out, outb, accumulate, alpha, U, s); break;
      case 2: splitk_direct_launch<2>(slabs, stride, n, out, outb, accumulate, alpha, U, s); break;
      case 3: splitk_direct_launch<3>(slabs, stride, n, out, outb, accumulate, alpha, U, s); break;
      case 4: splitk_direct_launch<4>(slabs, stride, n, out, outb, accumulate, alpha, U, s); break;
      case 5: splitk_direct_launch<5>(slabs, stride, n, out, outb, accumulate, alpha, U, s); break;
      case 6: splitk_direct_launch<6>(slabs, stride, n, out, outb, accumulate, alpha, U, s); break;
      case 7: splitk_direct_launch<7>(slabs, stride, n, out, outb, accumulate, alpha, U, s); break;
      default: splitk_direct_launch<8>(slabs, stride, n, out, outb, accumulate, alpha, U, s); break;
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
  const long long chunks = (n + 255) / 256;
  long long G = (1024 + chunks - 1) / chunks;
  const long long gmax = (S + 3) / 4;  // >= 4 slabs per group (one per wave)
  if (G > gmax) G = gmax;
  if (G > 64) G = 64;
  if (G < 1) G = 1;
  const int SG = (int)((S + G - 1) / G);
  G = (S + SG - 1) / SG;
  float* sl = const_cast<float*>(slabs);  // scratch: pass 1 parks group partials in place
  hipLaunchKernelGGL(splitk_partial_kernel, dim3((unsigned)chunks, (unsigned)G), dim3(256), 0, s, sl, S, SG, stride, n,
                     out, outb, accumulate, alpha);
  if (G > 1)
    hipLaunchKernelGGL(splitk_final_kernel, dim3((unsigned)((n + NT * 4 - 1) / (NT * 4))), dim3(NT), 0, s, slabs, (int)G,
                       SG, stride, n, out, outb, accumulate, alpha);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int tfk_transpose_arb(const bf16* in, bf16* out, int A, int R, int B, int flip, hipStream_t s) {
  dim3 grid((B + 31) / 32, (A + 31) / 32, R);
  hipLaunchKernelGGL(transpose_arb_kernel, grid, dim3(NT), 0, s, in, out, A, R, B, flip);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int tfk_transpose_f32(const float* in, float* out, int rows, int cols, hipStream_t s) {
  dim3 grid((cols + 31) / 32, (rows + 31) / 32);
  hipLaunchKernelGGL(transpose_f32_kernel, grid, dim3(NT), 0, s, in, out, rows, cols);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int tfk_cast_f32_bf16(const float* x, bf16* y, long long n, hipStream_t s) {
  long long done = 0;
  if ((((uintptr_t)x & 15) | ((uintptr_t)y & 7)) == 0 && n >= 4) {
    done = n / 4 * 4;
    hipLaunchKernelGGL(cast4_f32_bf16_kernel, dim3(grid_for(n / 4)), dim3(NT), 0, s, x, y, n / 4);
  }
  if (done < n)
    hipLaunchKernelGGL(cast_f32_bf16_kernel, dim3(grid_for(n - done)), dim3(NT), 0, s, x + done, y + done, n - done);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int tfk_cast_bf16_f32(const bf16* x, float* y, long long n, hipStream_t s) {
  long long done = 0;
  if ((((uintptr_t)x & 7) | ((uintptr_t)y & 15)) == 0 && n >= 4) {
    done = n / 4 * 4;
    hipLaunchKernelGGL(cast4_bf16_f32_kernel, dim3(grid_for(n / 4)), dim3(NT), 0, s, x, y, n / 4);
  }
  if (done < n)
    hipLaunchKernelGGL(cast_bf16_f32_kernel, dim3(grid_for(n - done)), dim3(NT), 0, s, x + done, y + done, n - done);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int tfk_synth_uniform(bf16* y, long long rows, int Creal, int Cpad, float lo, float hi, unsigned long long seed,
                      hipStream_t s) {
  hipLaunchKernelGGL(synth_uniform_kernel, dim3(grid_for(rows * Cpad)), dim3(NT), 0, s, y, rows, Creal, Cpad, lo, hi, seed);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int tfk_synth_normal_f32(float* y, long long n, float mean, float std, unsigned long long seed, hipStream_t s) {
  hipLaunchKernelGGL(synth_normal_f32_kernel, dim3(grid_for(n)), dim3(NT), 0, s, y, n, mean, std, seed);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int tfk_synth_labels(int* y, long long n, int classes, unsigned long long seed, hipStream_t s) {
  hipLaunchKernelGGL(synth_labels_kernel, dim3(grid_for(n)), dim3(NT), 0, s, y, n, classes, seed);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int tfk_colsum(const bf16* x, long long M, int N, long long ld, float* out, hipStream_t s) {
  if (N % 8 == 0 && ld % 8 == 0 && ((uintptr_t)x & 15) == 0) {
    static_assert(NT == 256, "colsum8 assumes 4 waves per block");
    const long long gx = (N + 511) / 512;
    long long gy = (M + 63) / 64;  // >= 16 rows per row group
    const long long cap = 2048 / gx > 0 ? 2048 / gx : 1;
    if (gy > cap) gy = cap;
    if (gy < 1) gy = 1;
    hipLaunchKernelGGL(colsum8_kernel, dim3((unsigned)gx, (unsigned)gy), dim3(NT), 0, s, x, M, N, ld, out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
  long long gy = (M + 255) / 256;
  if (gy > 1024) gy = 1024;
  if (gy < 1) gy = 1;
  dim3 grid((N + 63) / 64, (unsigned)gy);
  hipLaunchKernelGGL(colsum_kernel, grid, dim3(NT), 0, s, x, M, N, ld, out, 1);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int tfk_act_fwd(const bf16* x, const float* bias, int N, bf16* y, long long n, int act, hipStream_t s) {
  hipLaunchKernelGGL(act_fwd_kernel, dim3(grid_for(n)), dim3(NT), 0, s, x, bias, N, y, n, act);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int tfk_act_bwd(const bf16* dy, const bf16* x, bf16* dx, long long n, int act, hipStream_t s) {
  hipLaunchKernelGGL(act_bwd_kernel, dim3(grid_for(n)), dim3(NT), 0, s, dy, x, dx, n, act);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
// rng state [counter, key] (int64): counter += 1; key = splitmix64(counter ^ stream). One lane.
__global__ void rng_advance_kernel(unsigned long long* st, unsigned long long stream) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    const unsigned long long c = st[0] + 1;
    unsigned long long z = (c ^ stream) + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    st[0] = c;
    st[1] = z ^ (z >> 31);
  }
}

static const unsigned long long* g_seed_key = nullptr;
const unsigned long long* tfk_seed_key() { return g_seed_key; }
void tfk_set_seed_key(const unsigned long long* k) { g_seed_key = k; }
int tfk_rng_advance(unsigned long long* st, unsigned long long stream, hipStream_t s) {
  hipLaunchKernelGGL(rng_advance_kernel, dim3(1), dim3(64), 0, s, st, stream);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int tfk_dropout(const bf16* x, bf16* y, long long n, float p, unsigned long long seed, hipStream_t s) {
  if ((n & 7) == 0 && (((uintptr_t)x | (uintptr_t)y) & 15) == 0) {
    hipLaunchKernelGGL(dropout8_kernel, dim3(grid_for(n / 8)), dim3(NT), 0, s, x, y, n / 8, p, seed, tfk_seed_key());
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
  hipLaunchKernelGGL(dropout_kernel, dim3(grid_for(n)), dim3(NT), 0, s, x, y, n, p, seed, tfk_seed_key());
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int tfk_add(const bf16* a, const bf16* b, bf16* y, long long n, float alpha, float beta, hipStream_t s) {
  hipLaunchKernelGGL(add_kernel, dim3(grid_for(n)), dim3(NT), 0, s, a, b, y, n, alpha, beta);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
}
