// LayerNorm and embedding kernels for the transformer models (BERT, Transformer-big).
//
// LayerNorm over the last dim W (W % 8 == 0, W <= 2048): one wave64 per row, the row lives in
// registers (16-B bf16 vectors), exact two-pass mean/variance; saves mean and rstd (f32) for
// backward. Backward: dx = rstd*(g - mean(g) - xhat*mean(g*xhat)), g = dy*gamma, plus an optional
// residual-stream gradient added in the same pass; dgamma/dbeta are accumulated per lane across
// the rows a wave visits, reduced across the block in LDS, then one f32 atomic per column/block.
//
// Embedding: out[t] = word[ids[t]]*scale (+ pos[t % S]) (+ type[tt[t]]), 8 columns per thread.
// Backward: word rows by scattered f32 atomics (random ids rarely collide); position rows (hit by
// every sequence) by a plain batch reduction; token-type rows (2-4 rows hit by every token) by
// per-thread partial sums and one atomic per block -- no hot-row atomic contention.
#include "common.h"
#include "mx_common.h"

namespace {
constexpr int NT = 256;

template <int CPL>
__global__ __launch_bounds__(NT) void ln_fwd_kernel(const bf16* __restrict__ x, const float* __restrict__ gamma,
                                                    const float* __restrict__ beta, bf16* __restrict__ y,
                                                    float* __restrict__ mean, float* __restrict__ rstd, int M, int W,
                                                    float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (NT / 64) + (threadIdx.x >> 6);
  if (row >= M) return;
  const int nch = W >> 3;
  const bf16* xr = x + (long long)row * W;
  float v[CPL][8];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    const int c = lane + 64 * j;
    if (c < nch) {
      bf16x8 t = *(const bf16x8*)(xr + c * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) { v[j][e] = bf2f(t[e]); s += v[j][e]; }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[j][e] = 0.f;
    }
  }
  const float mu = wave_sum(s) / W;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < CPL; ++j)
    if (lane + 64 * j < nch)
#pragma unroll
      for (int e = 0; e < 8; ++e) { const float d = v[j][e] - mu; q += d * d; }
  const float rs = rsqrtf(wave_sum(q) / W + eps);
  bf16* yr = y + (long long)row * W;
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    const int c = lane + 64 * j;
    if (c < nch) {
      f32x4 g0 = *(const f32x4*)(gamma + c * 8), g1 = *(const f32x4*)(gamma + c * 8 + 4);
      f32x4 b0 = *(const f32x4*)(beta + c * 8), b1 = *(const f32x4*)(beta + c * 8 + 4);
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        o[e] = f2bf((v[j][e] - mu) * rs * g0[e] + b0[e]);
        o[e + 4] = f2bf((v[j][e + 4] - mu) * rs * g1[e] + b1[e]);
      }
      *(bf16x8*)(yr + c * 8) = o;
    }
  }
  if (lane == 0) { mean[row] = mu; rstd[row] = rs; }
}

// Width-specialized LayerNorm forward (W = 1024): ln_fwd_kernel's lane map and arithmetic
// (bit-identical outputs), but gamma / beta stay in registers across the rows of a grid-stride loop
// -- ln_fwd_kernel re-reads 8 B of them per element for every row, 4x the row's own bf16 bytes, from
// L2 -- and each iteration loads two rows before reducing either.
constexpr int LNF_ROWS = 4;  // rows per wave
template <int W>
__global__ __launch_bounds__(NT) void ln_fwd_fast_kernel(const bf16* __restrict__ x, const float* __restrict__ gamma,
                                                         const float* __restrict__ beta, bf16* __restrict__ y,
                                                         float* __restrict__ mean, float* __restrict__ rstd, int M,
                                                         float eps) {
  constexpr int NCH = W / 8, CPL = (NCH + 63) / 64;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float gm[CPL][8], bt[CPL][8];
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    const int c = lane + 64 * j;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      gm[j][e] = c < NCH ? gamma[c * 8 + e] : 0.f;
      bt[j][e] = c < NCH ? beta[c * 8 + e] : 0.f;
    }
  }
  auto load = [&](int r, bf16x8 (&t)[CPL]) {
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
      const int c = lane + 64 * j;
      if (c < NCH) t[j] = *(const bf16x8*)(x + (long long)r * W + c * 8);
    }
  };
  auto norm = [&](int r, const bf16x8 (&t)[CPL]) {
    float v[CPL][8];
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
      if (lane + 64 * j < NCH) {
#pragma unroll
        for (int e = 0; e < 8; ++e) { v[j][e] = bf2f(t[j][e]); s += v[j][e]; }
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[j][e] = 0.f;
      }
    }
    const float mu = wave_sum(s) / W;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < CPL; ++j)
      if (lane + 64 * j < NCH)
#pragma unroll
        for (int e = 0; e < 8; ++e) { const float d = v[j][e] - mu; q += d * d; }
    const float rs = rsqrtf(wave_sum(q) / W + eps);
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
      const int c = lane + 64 * j;
      if (c < NCH) {
        bf16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = f2bf((v[j][e] - mu) * rs * gm[j][e] + bt[j][e]);
        *(bf16x8*)(y + (long long)r * W + c * 8) = o;
      }
    }
    if (lane == 0) { mean[r] = mu; rstd[r] = rs; }
  };
  const int rstep = gridDim.x * (NT / 64);
  for (int row = blockIdx.x * (NT / 64) + wid; row < M; row += 2 * rstep) {
    const bool two = row + rstep < M;
    bf16x8 tA[CPL], tB[CPL];
    load(row, tA);
    if (two) load(row + rstep, tB);
    norm(row, tA);
    if (two) norm(row + rstep, tB);
  }
}

// LayerNorm forward that also emits both MX-fp8 quantizations of its output (the fp8 models' LN
// outputs feed only MX-fp8 GEMMs: the QKV / FFN-in / cross-attention projections and the tied
// logits): a block normalizes 32 rows (8 waves x 4 rows, same math as ln_fwd_kernel) into an LDS
// tile, then quantizes it in row blocks (qr [M][W], sr [M][W/32]) and column blocks of 32 rows
// (qc [W][M], sc [W][M/32]) -- the bytes of fp8.hip's dual quantizer without writing + re-reading
// the bf16 output (y may be null: no bf16 store). M % 32 == 0, W % 32 == 0, W <= 1024.
constexpr int LNMX_ROWS = 32, LNMX_NT = 512, LNMX_WMAX = 1024;
template <int CPL>
__global__ __launch_bounds__(LNMX_NT) void ln_fwd_mx_kernel(const bf16* __restrict__ x, const float* __restrict__ gamma,
                                                           const float* __restrict__ beta, bf16* __restrict__ y,
                                                           float* __restrict__ mean, float* __restrict__ rstd, int M, int W,
                                                           float eps, unsigned char* __restrict__ qr,
                                                           unsigned char* __restrict__ sr, unsigned char* __restrict__ qc,
                                                           unsigned char* __restrict__ sc) {
  __shared__ __attribute__((aligned(16))) bf16 tile[LNMX_ROWS][LNMX_WMAX + 8];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int r0 = blockIdx.x * LNMX_ROWS;
  const int nch = W >> 3;
  constexpr int RPW = LNMX_ROWS / (LNMX_NT / 64);
  // all RPW rows' loads issued up front (RPW x CPL 16-B vectors in flight per lane), then the
  // per-row reductions: one memory latency per wave instead of RPW
  bf16x8 raw[RPW][CPL];
#pragma unroll
  for (int rr = 0; rr < RPW; ++rr) {
    const bf16* xr = x + (long long)(r0 + wv * RPW + rr) * W;
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
      const int c = lane + 64 * j;
      if (c < nch) raw[rr][j] = *(const bf16x8*)(xr + c * 8);
    }
  }
#pragma unroll
  for (int rr = 0; rr < RPW; ++rr) {
    const int lr = wv * RPW + rr, row = r0 + lr;
    float v[CPL][8];
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
      const int c = lane + 64 * j;
      if (c < nch) {
#pragma unroll
        for (int e = 0; e < 8; ++e) { v[j][e] = bf2f(raw[rr][j][e]); s += v[j][e]; }
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[j][e] = 0.f;
      }
    }
    const float mu = wave_sum(s) / W;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < CPL; ++j)
      if (lane + 64 * j < nch)
#pragma unroll
        for (int e = 0; e < 8; ++e) { const float d = v[j][e] - mu; q += d * d; }
    const float rs = rsqrtf(wave_sum(q) / W + eps);
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
      const int c = lane + 64 * j;
      if (c < nch) {
        f32x4 g0 = *(const f32x4*)(gamma + c * 8), g1 = *(const f32x4*)(gamma + c * 8 + 4);
        f32x4 b0 = *(const f32x4*)(beta + c * 8), b1 = *(const f32x4*)(beta + c * 8 + 4);
        bf16x8 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          o[e] = f2bf((v[j][e] - mu) * rs * g0[e] + b0[e]);
          o[e + 4] = f2bf((v[j][e + 4] - mu) * rs * g1[e] + b1[e]);
        }
        *(bf16x8*)&tile[lr][c * 8] = o;
        if (y) *(bf16x8*)(y + (long long)row * W + c * 8) = o;
      }
    }
    if (lane == 0) { mean[row] = mu; rstd[row] = rs; }
  }
  __syncthreads();
  tfk::mx_rows32_out<LNMX_NT>(&tile[0][0], LNMX_WMAX + 8, W, M, r0, qr, sr, qc, sc);
}

// Per-element arithmetic of the LayerNorm backward, spelled out with explicit rounding and no
// compiler contraction (shared by ln_bwd_kernel and ln_bwd_fast_kernel).
__device__ __forceinline__ void ln_bwd_accum(float d, float xv, float mu, float rs, float gmv, float& g, float& xh,
                                             float& s1, float& s2, float& dgv, float& dbv) {
#pragma clang fp contract(off)
  xh = __fmul_rn(__fsub_rn(xv, mu), rs);
  g = __fmul_rn(d, gmv);
  s1 = __fadd_rn(s1, g);
  s2 = __fmaf_rn(g, xh, s2);
  dgv = __fmaf_rn(d, xh, dgv);
  dbv = __fadd_rn(dbv, d);
}
__device__ __forceinline__ float ln_bwd_out(float g, float xh, float s1, float s2, float rs, float res) {
#pragma clang fp contract(off)
  return __fadd_rn(__fmul_rn(rs, __fmaf_rn(-xh, s2, __fsub_rn(g, s1))), res);
}

template <int CPL>
__global__ __launch_bounds__(NT) void ln_bwd_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ x,
                                                    const float* __restrict__ gamma, const float* __restrict__ mean,
                                                    const float* __restrict__ rstd, const bf16* __restrict__ dres,
                                                    bf16* __restrict__ dx, float* __restrict__ dgamma,
                                                    float* __restrict__ dbeta, int M, int W, bf16* __restrict__ dxd,
                                                    float drop_p, unsigned long long drop_salt,
                                                    const unsigned long long* __restrict__ drop_key,
                                                    float* __restrict__ dbias, unsigned char* __restrict__ mq,
                                                    unsigned char* __restrict__ ms, unsigned char* __restrict__ mqt,
                                                    unsigned char* __restrict__ mst, float* __restrict__ part) {
  // dbias (optional): += column sums of the gradient this kernel hands its consumer (dxd, else dx)
  // -- that Linear's bias gradient, reduced with dgamma/dbeta instead of a separate column-sum pass
  extern __shared__ float red[];  // [NT/64][2 or 3][W]
  const int NS = dbias ? 3 : 2;
  const unsigned long long drop_seed = eff_seed(drop_salt, drop_key);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nch = W >> 3;
  float dg[CPL][8], db[CPL][8], gm[CPL][8], bs[CPL][8];
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    const int c = lane + 64 * j;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      dg[j][e] = 0.f; db[j][e] = 0.f; bs[j][e] = 0.f;
      gm[j][e] = c < nch ? gamma[c * 8 + e] : 0.f;
    }
  }
  // rows software-pipelined: the next row's dy / x / dres (and mean / rstd) are loaded before this
  // row's reductions and stores, so a wave keeps one row of loads in flight instead of paying two
  // dependent memory latencies per row (measured 2.2 TB/s on Transformer-big's 8192 x 1024 rows)
  // MX mode (mq != null: emit MX-fp8 row + column blocks of the consumer gradient): a block owns 32
  // consecutive rows (8 per wave), stages their final values in an LDS tile behind `red` and
  // quantizes the tile after the row loop (the consumer's fp8 backward then skips its quantize pass)
  const bool mxo = mq != nullptr;
  const int rstep = mxo ? 1 : gridDim.x * (NT / 64);
  int row = mxo ? blockIdx.x * 32 + wid * 8 : blockIdx.x * (NT / 64) + wid;
  const int rend = mxo ? row + 8 : M;
  bf16* mtile = (bf16*)(red + (NT / 64) * NS * W);  // [32][W + 8] (MX mode only)
  bf16x8 ndv[CPL], nxv[CPL], nrv[CPL];
  float nmu = 0.f, nrs = 0.f;
  auto fetch = [&](int r) {
    nmu = mean[r];
    nrs = rstd[r];
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
      const int c = lane + 64 * j;
      if (c < nch) {
        ndv[j] = *(const bf16x8*)(dy + (long long)r * W + c * 8);
        nxv[j] = *(const bf16x8*)(x + (long long)r * W + c * 8);
        if (dres) nrv[j] = *(const bf16x8*)(dres + (long long)r * W + c * 8);
      }
    }
  };
  if (row < rend) fetch(row);
  for (; row < rend; row += rstep) {
    const float mu = nmu, rs = nrs;
    bf16x8 cdv[CPL], cxv[CPL], crv[CPL];
#pragma unroll
    for (int j = 0; j < CPL; ++j) { cdv[j] = ndv[j]; cxv[j] = nxv[j]; crv[j] = nrv[j]; }
    if (row + rstep < rend) fetch(row + rstep);
    float g[CPL][8], xh[CPL][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
      const int c = lane + 64 * j;
      if (c < nch) {
        const bf16x8 dv = cdv[j], xv = cxv[j];
#pragma unroll
        for (int e = 0; e < 8; ++e)
          ln_bwd_accum(bf2f(dv[e]), bf2f(xv[e]), mu, rs, gm[j][e], g[j][e], xh[j][e], s1, s2, dg[j][e], db[j][e]);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) { g[j][e] = 0.f; xh[j][e] = 0.f; }
      }
    }
    s1 = wave_sum(s1) / W;
    s2 = wave_sum(s2) / W;
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
      const int c = lane + 64 * j;
      if (c < nch) {
        const bf16x8 rv = crv[j];
        bf16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          o[e] = f2bf(ln_bwd_out(g[j][e], xh[j][e], s1, s2, rs, dres ? bf2f(rv[e]) : 0.f));
        }
        *(bf16x8*)(dx + (long long)row * W + c * 8) = o;
        if (dxd) {
          // the consumer's dropout backward on the stored dx (misc.hip dropout_kernel's mask and
          // arithmetic, index row*W + col): saves that pass's read + write of dx
          const float inv = drop_scale8(drop_p);
          const unsigned long long base = (unsigned long long)row * W + c * 8;
          const unsigned km = drop_keep8(drop_seed32(drop_seed), base, drop_thr8(drop_p));
          bf16x8 od;
#pragma unroll
          for (int e = 0; e < 8; ++e) od[e] = f2bf((km >> e) & 1u ? bf2f(o[e]) * inv : 0.f);
          *(bf16x8*)(dxd + base) = od;
          if (dbias) {
#pragma unroll
            for (int e = 0; e < 8; ++e) bs[j][e] += bf2f(od[e]);
          }
          if (mxo) *(bf16x8*)(mtile + (row - blockIdx.x * 32) * (W + 8) + c * 8) = od;
        } else {
          if (dbias) {
#pragma unroll
            for (int e = 0; e < 8; ++e) bs[j][e] += bf2f(o[e]);
          }
          if (mxo) *(bf16x8*)(mtile + (row - blockIdx.x * 32) * (W + 8) + c * 8) = o;
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    const int c = lane + 64 * j;
    if (c < nch)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        red[(wid * NS + 0) * W + c * 8 + e] = dg[j][e];
        red[(wid * NS + 1) * W + c * 8 + e] = db[j][e];
        if (dbias) red[(wid * NS + 2) * W + c * 8 + e] = bs[j][e];
      }
  }
  __syncthreads();
  // block partials: plain stores into this block's slab row (part), reduced by ln_part_reduce_kernel
  // -- every block adding atomically into the same 2-3 x W floats serialised on those few lines at
  // the kernel's tail (256 adders per address on Transformer-big's 8192 rows)
  float* prow = part ? part + (long long)blockIdx.x * NS * W : nullptr;
  for (int col = threadIdx.x; col < W; col += NT) {
    float a = 0.f, b2 = 0.f, b3 = 0.f;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) {
      a += red[(w * NS) * W + col];
      b2 += red[(w * NS + 1) * W + col];
      if (dbias) b3 += red[(w * NS + 2) * W + col];
    }
    if (prow) {
      prow[col] = a;
      prow[W + col] = b2;
      if (dbias) prow[2 * W + col] = b3;
    } else {
      atomicAdd(dgamma + col, a);
      atomicAdd(dbeta + col, b2);
      if (dbias) atomicAdd(dbias + col, b3);
    }
  }
  if (mxo) tfk::mx_rows32_out<NT>(mtile, W + 8, W, M, blockIdx.x * 32, mq, ms, mqt, mst);  // tile complete: barrier above
}

// Column sums of the ln_bwd block partials part[nblk][NS][W] into dgamma / dbeta / dbias (added):
// grid.y row groups of the slabs each sum their share and add it with one atomic per column
// (LN_PART_GROUPS adders per address instead of one per block). 32 groups of <= 8 slabs with the 8
// loads of a group in flight together: 8 groups of 32 slabs walked one load at a time measured
// 9.4 us per call on Transformer-big (256 slabs x 2 x 1024: a latency chain, 0.3 TB/s).
// Width-specialized LayerNorm backward (bf16 mode, W = 256 * Q4: BERT-base 768, Transformer-big /
// BERT-large 1024). PMC of ln_bwd_kernel (profiles/pmc_ln_bwd_r6.txt): ~37 VALU instructions per
// element -- per-lane chunk guards, runtime option branches, 64-bit index math and register copies
// of the prefetched row -- against ~13 the arithmetic needs, at one wave per SIMD: VALU issue and
// memory waits did not overlap (22.5 us for the 48 MB of a plain 8192 x 1024 call). Here width and
// options are compile-time, lane l owns the 4-element chunks l + 64 q (q < Q4; every 8-B load of a
// wave is a contiguous 512 B), and each iteration loads two rows before using either. (The generic
// kernel's 8-element lane map measured 22.1 vs 19.2 us on BERT-base's call form.)
template <int Q4, bool DRES, bool DROP, bool DBIAS>
__global__ __launch_bounds__(NT) void ln_bwd_fast_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ x,
                                                         const float* __restrict__ gamma, const float* __restrict__ mean,
                                                         const float* __restrict__ rstd, const bf16* __restrict__ dres,
                                                         bf16* __restrict__ dx, float* __restrict__ dgamma,
                                                         float* __restrict__ dbeta, int M, bf16* __restrict__ dxd,
                                                         float drop_p, unsigned long long drop_salt,
                                                         const unsigned long long* __restrict__ drop_key,
                                                         float* __restrict__ dbias, float* __restrict__ part) {
  constexpr int W = 256 * Q4, NS = DBIAS ? 3 : 2;
  extern __shared__ float red[];  // [NT/64][NS][W]
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float gm[Q4][4], dg[Q4][4], db[Q4][4], bs[Q4][4];
#pragma unroll
  for (int q = 0; q < Q4; ++q) {
    const f32x4 g4 = *(const f32x4*)(gamma + lane * 4 + 256 * q);
#pragma unroll
    for (int e = 0; e < 4; ++e) { gm[q][e] = g4[e]; dg[q][e] = 0.f; db[q][e] = 0.f; bs[q][e] = 0.f; }
  }
  const uint32_t s32 = DROP ? drop_seed32(eff_seed(drop_salt, drop_key)) : 0u;
  const uint32_t thr = DROP ? (uint32_t)drop_thr8(drop_p) : 0u;
  const float inv = DROP ? drop_scale8(drop_p) : 1.f;
  auto load_row = [&](int r, bf16x4 (&dv)[Q4], bf16x4 (&xv)[Q4], bf16x4 (&rv)[Q4]) {
    const long long base = (long long)r * W + lane * 4;
#pragma unroll
    for (int q = 0; q < Q4; ++q) {
      dv[q] = *(const bf16x4*)(dy + base + 256 * q);
      xv[q] = *(const bf16x4*)(x + base + 256 * q);
      if constexpr (DRES) rv[q] = *(const bf16x4*)(dres + base + 256 * q);
    }
  };
  auto do_row = [&](int r, float mu, float rs, const bf16x4 (&dv)[Q4], const bf16x4 (&xv)[Q4], const bf16x4 (&rv)[Q4]) {
    float g[Q4][4], xh[Q4][4];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int q = 0; q < Q4; ++q)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        ln_bwd_accum(bf2f(dv[q][e]), bf2f(xv[q][e]), mu, rs, gm[q][e], g[q][e], xh[q][e], s1, s2, dg[q][e], db[q][e]);
    s1 = wave_sum(s1) / W;
    s2 = wave_sum(s2) / W;
    const long long base = (long long)r * W + lane * 4;
#pragma unroll
    for (int q = 0; q < Q4; ++q) {
      bf16x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = f2bf(ln_bwd_out(g[q][e], xh[q][e], s1, s2, rs, DRES ? bf2f(rv[q][e]) : 0.f));
      *(bf16x4*)(dx + base + 256 * q) = o;
      if constexpr (DROP) {
        // the consumer's dropout backward: misc.hip's mask (one hash per 4 elements, byte e of
        // hash32(s32 ^ idx / 4) against the 8-bit threshold) on index r * W + col
        const uint32_t h = hash32(s32 ^ (uint32_t)((base + 256 * q) >> 2));
        bf16x4 od;
#pragma unroll
        for (int e = 0; e < 4; ++e) od[e] = f2bf(((h >> (8 * e)) & 0xffu) >= thr ? bf2f(o[e]) * inv : 0.f);
        *(bf16x4*)(dxd + base + 256 * q) = od;
        if constexpr (DBIAS) {
#pragma unroll
          for (int e = 0; e < 4; ++e) bs[q][e] += bf2f(od[e]);
        }
      } else if constexpr (DBIAS) {
#pragma unroll
        for (int e = 0; e < 4; ++e) bs[q][e] += bf2f(o[e]);
      }
    }
  };
  const int rstep = gridDim.x * (NT / 64);
  for (int row = blockIdx.x * (NT / 64) + wid; row < M; row += 2 * rstep) {
    const bool two = row + rstep < M;
    const int r1 = two ? row + rstep : row;
    bf16x4 dA[Q4], xA[Q4], rA[Q4], dB[Q4], xB[Q4], rB[Q4];
    const float muA = mean[row], rsA = rstd[row], muB = mean[r1], rsB = rstd[r1];
    load_row(row, dA, xA, rA);
    load_row(r1, dB, xB, rB);
    do_row(row, muA, rsA, dA, xA, rA);
    if (two) do_row(r1, muB, rsB, dB, xB, rB);
  }
#pragma unroll
  for (int q = 0; q < Q4; ++q) {
    const int c = lane * 4 + 256 * q;
    *(f32x4*)(red + (wid * NS + 0) * W + c) = f32x4{dg[q][0], dg[q][1], dg[q][2], dg[q][3]};
    *(f32x4*)(red + (wid * NS + 1) * W + c) = f32x4{db[q][0], db[q][1], db[q][2], db[q][3]};
    if constexpr (DBIAS) *(f32x4*)(red + (wid * NS + 2) * W + c) = f32x4{bs[q][0], bs[q][1], bs[q][2], bs[q][3]};
  }
  __syncthreads();
  float* prow = part ? part + (long long)blockIdx.x * NS * W : nullptr;
  for (int col = threadIdx.x; col < W; col += NT) {
    float a = 0.f, b2 = 0.f, b3 = 0.f;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) {
      a += red[(w * NS) * W + col];
      b2 += red[(w * NS + 1) * W + col];
      if constexpr (DBIAS) b3 += red[(w * NS + 2) * W + col];
    }
    if (prow) {
      prow[col] = a;
      prow[W + col] = b2;
      if constexpr (DBIAS) prow[2 * W + col] = b3;
    } else {
      atomicAdd(dgamma + col, a);
      atomicAdd(dbeta + col, b2);
      if constexpr (DBIAS) atomicAdd(dbias + col, b3);
    }
  }
}

constexpr int LN_PART_GROUPS = 32;
__global__ void ln_part_reduce_kernel(const float* __restrict__ part, int nblk, int NS, int W, float* __restrict__ dgamma,
                                      float* __restrict__ dbeta, float* __restrict__ dbias) {
  const int c = blockIdx.x * NT + threadIdx.x;
  if (c >= NS * W) return;
  const int per = (nblk + gridDim.y - 1) / gridDim.y, b0 = blockIdx.y * per, b1 = min(nblk, b0 + per);
  float v = 0.f;
#pragma unroll 8
  for (int b = b0; b < b1; ++b) v += part[(long long)b * NS * W + c];
  const int which = c / W, col = c - which * W;
  atomicAdd((which == 0 ? dgamma : which == 1 ? dbeta : dbias) + col, v);
}

__global__ void embed_fwd_kernel(const int* __restrict__ ids, const bf16* __restrict__ word, int V,
                                 const bf16* __restrict__ pos, int S, const int* __restrict__ tt,
                                 const bf16* __restrict__ type, int T, bf16* __restrict__ out, long long ntok, int W,
                                 float scale) {
  const int cpr = W >> 3;
  const long long n = ntok * cpr;
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) {
    const long long t = i / cpr;
    const int c = (int)(i - t * cpr) * 8;
    const int id = min(max(ids[t], 0), V - 1);
    bf16x8 wv = *(const bf16x8*)(word + (long long)id * W + c);
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = bf2f(wv[e]) * scale;
    if (pos) {
      bf16x8 pv = *(const bf16x8*)(pos + (long long)(t % S) * W + c);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] += bf2f(pv[e]);
    }
    if (type) {
      const int ty = min(max(tt[t], 0), T - 1);
      bf16x8 tv = *(const bf16x8*)(type + (long long)ty * W + c);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] += bf2f(tv[e]);
    }
    bf16x8 r;
#pragma unroll
    for (int e = 0; e < 8; ++e) r[e] = f2bf(o[e]);
    *(bf16x8*)(out + t * W + c) = r;
  }
}

// word rows: scattered f32 atomics (token ids rarely collide)
__global__ void embed_bwd_kernel(const int* __restrict__ ids, const bf16* __restrict__ dy, int V,
                                 float* __restrict__ dword, long long ntok, int W, float scale) {
  const int cpr = W >> 3;
  const long long n = ntok * cpr;
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) {
    const long long t = i / cpr;
    const int c = (int)(i - t * cpr) * 8;
    bf16x8 g = *(const bf16x8*)(dy + t * W + c);
    const int id = min(max(ids[t], 0), V - 1);
    float* dw = dword + (long long)id * W + c;
#pragma unroll
    for (int e = 0; e < 8; ++e) atomicAdd(dw + e, bf2f(g[e]) * scale);
  }
}

// Word-row gradient without per-element atomics: tokens are bucketed by row (count -> scan ->
// scatter, int atomics only), then one block per touched row sums its tokens' dy rows in f32 and adds
// the result to the row once. The scattered f32 atomics (8192 tokens x 1024 columns) ran at
// ~37 G atomics/s: 223 us per call on Transformer-big's tied 33792 x 1024 table.
// Out-of-range events of the bucketed backward (a corrupted count / cursor): the kernels skip the
// access instead of faulting and count it here (tfk_emb_guard_count reads and clears it).
__device__ int g_emb_guard = 0;
__global__ void emb_zero_kernel(int* __restrict__ p, int n) {
  for (int i = blockIdx.x * NT + threadIdx.x; i < n; i += gridDim.x * NT) p[i] = 0;
}
__global__ void emb_count_kernel(const int* __restrict__ ids, long long ntok, int V, int* __restrict__ cnt) {
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < ntok; i += (long long)gridDim.x * NT)
    atomicAdd(cnt + min(max(ids[i], 0), V - 1), 1);
}
// exclusive scan cnt[V] -> off[V] (and cursor = off): one 1024-thread block walking the counts in
// coalesced 1024-element chunks (every chunk's load issued before any scan, so the V/1024 global
// latencies overlap instead of chaining), each chunk scanned with DPP/permlane wave prefix sums and a
// 16-entry cross-wave pass. (The previous form -- a thread per contiguous segment, loads in a runtime
// loop -- serialised ~66 dependent global loads per thread: 67 us per call on the 33728-row table.)
constexpr int EMB_SCAN_CH = 40;  // chunks held in registers (V <= 40960); larger V loops in groups
__device__ __forceinline__ int wave_incl_scan(int v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_up(v, o, 64);
    if (lane >= o) v += u;
  }
  return v;
}
__global__ __launch_bounds__(1024) void emb_scan_kernel(const int* __restrict__ cnt, int V, int* __restrict__ off,
                                                        int* __restrict__ cursor) {
  __shared__ int wsum[16];
  __shared__ int carry_s;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  if (t == 0) carry_s = 0;
  __syncthreads();
  for (int g0 = 0; g0 < V; g0 += EMB_SCAN_CH * 1024) {
    int v[EMB_SCAN_CH];
#pragma unroll
    for (int c = 0; c < EMB_SCAN_CH; ++c) {
      const int i = g0 + c * 1024 + t;
      v[c] = i < V ? cnt[i] : 0;
    }
#pragma unroll
    for (int c = 0; c < EMB_SCAN_CH; ++c) {
      if (g0 + c * 1024 >= V) break;  // block-uniform
      const int x = v[c];
      const int inc = wave_incl_scan(x);
      if (lane == 63) wsum[w] = inc;
      __syncthreads();
      int before = carry_s, tot = 0;
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int s = wsum[k];
        before += k < w ? s : 0;
        tot += s;
      }
      const int i = g0 + c * 1024 + t;
      if (i < V) {
        const int ex = before + inc - x;
        off[i] = ex;
        cursor[i] = ex;
      }
      __syncthreads();  // every wave read wsum / carry_s before they change
      if (t == 0) carry_s += tot;
      __syncthreads();
    }
  }
}
__global__ void emb_bucket_kernel(const int* __restrict__ ids, long long ntok, int V, int* __restrict__ cursor,
                                  int* __restrict__ list) {
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < ntok; i += (long long)gridDim.x * NT) {
    const int pos = atomicAdd(cursor + min(max(ids[i], 0), V - 1), 1);
    if ((unsigned long long)pos < (unsigned long long)ntok) list[pos] = (int)i;
    else atomicAdd(&g_emb_guard, 1);
  }
}
// one block per vocab row: dword[row] += scale * sum over the row's tokens of dy[token] (f32)
__global__ void emb_reduce_kernel(const int* __restrict__ off, const int* __restrict__ cnt, const int* __restrict__ list,
                                  const bf16* __restrict__ dy, float* __restrict__ dword, int W, float scale,
                                  long long ntok) {
  const int row = blockIdx.x, n = cnt[row];
  if (n == 0) return;
  const int o = off[row];
  if (n < 0 || o < 0 || (long long)o + n > ntok) {
    if (threadIdx.x == 0) atomicAdd(&g_emb_guard, 1);
    return;
  }
  const int* lst = list + o;
  for (int c = threadIdx.x * 8; c < W; c += NT * 8) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < n; ++k) {
      const int tok = lst[k];
      if ((unsigned long long)tok >= (unsigned long long)ntok) continue;  // (never for consistent counts)
      const bf16x8 g = *(const bf16x8*)(dy + (long long)tok * W + c);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += bf2f(g[e]);
    }
    float* dw = dword + (long long)row * W + c;
    const f32x4 a = *(const f32x4*)dw, b = *(const f32x4*)(dw + 4);
    *(f32x4*)dw = f32x4{a[0] + acc[0] * scale, a[1] + acc[1] * scale, a[2] + acc[2] * scale, a[3] + acc[3] * scale};
    *(f32x4*)(dw + 4) = f32x4{b[0] + acc[4] * scale, b[1] + acc[5] * scale, b[2] + acc[6] * scale, b[3] + acc[7] * scale};
  }
}

// position rows: every sequence hits every row -> a plain column reduction over the batch
// (deterministic, no atomics). Thread = (position s, 8-column chunk).
__global__ void embed_pos_bwd_kernel(const bf16* __restrict__ dy, float* __restrict__ dpos, int S, int nseq, int W) {
  const int cpr = W >> 3;
  const long long n = (long long)S * cpr;
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) {
    const int s = (int)(i / cpr), c = (int)(i % cpr) * 8;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int b = 0; b < nseq; ++b) {
      bf16x8 g = *(const bf16x8*)(dy + ((long long)b * S + s) * W + c);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += bf2f(g[e]);
    }
    *(f32x4*)(dpos + (long long)s * W + c) = f32x4{acc[0], acc[1], acc[2], acc[3]};
    *(f32x4*)(dpos + (long long)s * W + c + 4) = f32x4{acc[4], acc[5], acc[6], acc[7]};
  }
}

// token-type rows (T <= 4): per-thread partial sums over a token range, one atomic per block.
__global__ void embed_type_bwd_kernel(const bf16* __restrict__ dy, const int* __restrict__ tt, float* __restrict__ dtype,
                                      int T, long long ntok, int W) {
  const int cpr = W >> 3;
  const long long per = (ntok + gridDim.y - 1) / gridDim.y;
  const long long t0 = (long long)blockIdx.y * per, t1 = min(ntok, t0 + per);
  for (int c8 = blockIdx.x * NT + threadIdx.x; c8 < cpr; c8 += gridDim.x * NT) {
    float acc[4][8];
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[k][e] = 0.f;
    for (long long t = t0; t < t1; ++t) {
      const int ty = min(max(tt[t], 0), T - 1);
      bf16x8 g = *(const bf16x8*)(dy + t * W + c8 * 8);
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (k == ty)
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[k][e] += bf2f(g[e]);
    }
    for (int k = 0; k < T; ++k)
#pragma unroll
      for (int e = 0; e < 8; ++e) atomicAdd(dtype + (long long)k * W + c8 * 8 + e, acc[k][e]);
  }
}

int grid_for(long long work, int per_block, int cap) {
  long long g = (work + per_block - 1) / per_block;
  return (int)(g < 1 ? 1 : (g > cap ? cap : g));
}
template <int Q4>
void ln_bwd_fast_launch(dim3 grid, size_t sh, hipStream_t s, const bf16* dy, const bf16* x, const float* gamma,
                               const float* mean, const float* rstd, const bf16* dres, bf16* dx, float* dgamma,
                               float* dbeta, int M, bf16* dxd, float drop_p, unsigned long long drop_seed, float* dbias,
                               float* part) {
#define TFK_LNF(R_, D_, B_)                                                                                       \
  if ((dres != nullptr) == R_ && (dxd != nullptr) == D_ && (dbias != nullptr) == B_) {                            \
    hipLaunchKernelGGL((ln_bwd_fast_kernel<Q4, R_, D_, B_>), grid, dim3(NT), sh, s, dy, x, gamma, mean, rstd, dres, dx, \
                       dgamma, dbeta, M, dxd, drop_p, drop_seed, tfk_seed_key(), dbias, part);                      \
    return;                                                                                                      \
  }
  TFK_LNF(false, false, false) TFK_LNF(false, false, true) TFK_LNF(false, true, false) TFK_LNF(false, true, true)
  TFK_LNF(true, false, false) TFK_LNF(true, false, true) TFK_LNF(true, true, false) TFK_LNF(true, true, true)
#undef TFK_LNF
}
}  // namespace

extern "C" {
// W = 1024 forwards on ln_fwd_fast_kernel (A/B knob; TFK_LN_FWD_FAST=0 disables)
static int g_ln_fwd_fast = -1;
void tfk_ln_fwd_set_fast(int on) { g_ln_fwd_fast = on ? 1 : 0; }
static bool ln_fwd_fast() {
  if (g_ln_fwd_fast < 0) {
    const char* e = getenv("TFK_LN_FWD_FAST");
    g_ln_fwd_fast = (e && e[0] == '0') ? 0 : 1;
  }
  return g_ln_fwd_fast == 1;
}
int tfk_layernorm_fwd(const bf16* x, const float* gamma, const float* beta, bf16* y, float* mean, float* rstd, int M,
                      int W, float eps, hipStream_t s) {
  const int cpl = (W / 8 + 63) / 64;
  // W = 1024 only: at 768 (half the lanes idle on the second chunk) it measured slower than
  // ln_fwd_kernel (7.8 vs 6.7 us for 8192 rows; 1024: 6.5 vs 7.6)
  if (W == 1024 && ln_fwd_fast() && ((((uintptr_t)x | (uintptr_t)y) & 15) == 0)) {
    dim3 g((unsigned)((M + (NT / 64) * LNF_ROWS - 1) / ((NT / 64) * LNF_ROWS)));
    hipLaunchKernelGGL(ln_fwd_fast_kernel<1024>, g, dim3(NT), 0, s, x, gamma, beta, y, mean, rstd, M, eps);
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
  dim3 grid((M + NT / 64 - 1) / (NT / 64));
  if (cpl <= 1) hipLaunchKernelGGL(ln_fwd_kernel<1>, grid, dim3(NT), 0, s, x, gamma, beta, y, mean, rstd, M, W, eps);
  else if (cpl <= 2) hipLaunchKernelGGL(ln_fwd_kernel<2>, grid, dim3(NT), 0, s, x, gamma, beta, y, mean, rstd, M, W, eps);
  else if (cpl <= 4) hipLaunchKernelGGL(ln_fwd_kernel<4>, grid, dim3(NT), 0, s, x, gamma, beta, y, mean, rstd, M, W, eps);
  else return -3;
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
// y may be null (MX outputs only); qr/sr/qc/sc: MX row / column block outputs (ln_fwd_mx_kernel)
int tfk_layernorm_fwd_mx(const bf16* x, const float* gamma, const float* beta, bf16* y, float* mean, float* rstd, int M,
                         int W, float eps, void* qr, void* sr, void* qc, void* sc, hipStream_t s) {
  if (M % LNMX_ROWS || W % 32 || W > LNMX_WMAX) return -3;
  const int cpl = (W / 8 + 63) / 64;
  dim3 grid(M / LNMX_ROWS);
  auto* q0 = (unsigned char*)qr; auto* s0 = (unsigned char*)sr; auto* q1 = (unsigned char*)qc; auto* s1 = (unsigned char*)sc;
  if (cpl <= 1)
    hipLaunchKernelGGL(ln_fwd_mx_kernel<1>, grid, dim3(LNMX_NT), 0, s, x, gamma, beta, y, mean, rstd, M, W, eps, q0, s0, q1, s1);
  else
    hipLaunchKernelGGL(ln_fwd_mx_kernel<2>, grid, dim3(LNMX_NT), 0, s, x, gamma, beta, y, mean, rstd, M, W, eps, q0, s0, q1, s1);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
// dxd (optional): also write dropout(dx; drop_p, drop_seed) -- the gradient the consumer's dropout
// backward would produce from dx
// blocks of the LayerNorm-backward grid (the binding sizes the partials workspace with it)
// bf16 mode: rows per wave of the grid-stride backward (A/B knob of tools/ln_probe.py; fewer rows per
// wave = more blocks per CU in flight, more column-partial slabs for ln_part_reduce_kernel)
// (TFK_LN_ROWS sets the starting value, default 8)
static int g_ln_rows = -1;
void tfk_ln_bwd_set_rows(int r) { g_ln_rows = r > 0 ? r : 8; }
static int ln_rows() {
  if (g_ln_rows < 0) {
    const char* e = getenv("TFK_LN_ROWS");
    const int r = e ? atoi(e) : 0;
    g_ln_rows = r > 0 ? r : 8;
  }
  return g_ln_rows;
}
// bf16-mode calls at W = 768 / 1024 on ln_bwd_fast_kernel (A/B knob; TFK_LN_FAST=0 disables)
static int g_ln_fast = -1;
void tfk_ln_bwd_set_fast(int on) { g_ln_fast = on ? 1 : 0; }
static bool ln_fast() {
  if (g_ln_fast < 0) {
    const char* e = getenv("TFK_LN_FAST");
    g_ln_fast = (e && e[0] == '0') ? 0 : 1;
  }
  return g_ln_fast == 1;
}

int tfk_ln_bwd_blocks(int M, int mxo) { return mxo ? M / 32 : (int)grid_for(M, (NT / 64) * ln_rows(), 4096); }
static unsigned ln_bwd_blocks(int M, bool mxo) { return (unsigned)tfk_ln_bwd_blocks(M, mxo ? 1 : 0); }
// part (optional): f32 workspace [blocks][2 or 3][W] for the column partials (no tail atomics)
int tfk_layernorm_bwd(const bf16* dy, const bf16* x, const float* gamma, const float* mean, const float* rstd,
                      const bf16* dres, bf16* dx, float* dgamma, float* dbeta, int M, int W, bf16* dxd, float drop_p,
                      unsigned long long drop_seed, float* dbias, void* mq, void* ms, void* mqt, void* mst,
                      float* part, hipStream_t s) {
  const int cpl = (W / 8 + 63) / 64;
  const bool mxo = mq != nullptr;
  if (mxo && (M % 32 || W % 32 || W > 1024)) return -3;
  dim3 grid(ln_bwd_blocks(M, mxo));
  const size_t sh = (size_t)(NT / 64) * (dbias ? 3 : 2) * W * sizeof(float) + (mxo ? (size_t)32 * (W + 8) * 2 : 0);
  const bool aligned = ((((uintptr_t)dy | (uintptr_t)x | (uintptr_t)dx | (uintptr_t)(dres ? dres : dy) |
                          (uintptr_t)(dxd ? dxd : dx)) & 7) == 0) && ((uintptr_t)gamma & 15) == 0;
  if (!mxo && aligned && (W == 768 || W == 1024) && ln_fast()) {
    if (W == 768)
      ln_bwd_fast_launch<3>(grid, sh, s, dy, x, gamma, mean, rstd, dres, dx, dgamma, dbeta, M, dxd, drop_p, drop_seed,
                            dbias, part);
    else
      ln_bwd_fast_launch<4>(grid, sh, s, dy, x, gamma, mean, rstd, dres, dx, dgamma, dbeta, M, dxd, drop_p, drop_seed,
                            dbias, part);
  } else if (cpl <= 1)
    hipLaunchKernelGGL(ln_bwd_kernel<1>, grid, dim3(NT), sh, s, dy, x, gamma, mean, rstd, dres, dx, dgamma, dbeta, M, W,
                       dxd, drop_p, drop_seed, tfk_seed_key(), dbias, (unsigned char*)mq, (unsigned char*)ms,
                       (unsigned char*)mqt, (unsigned char*)mst, part);
  else if (cpl <= 2)
    hipLaunchKernelGGL(ln_bwd_kernel<2>, grid, dim3(NT), sh, s, dy, x, gamma, mean, rstd, dres, dx, dgamma, dbeta, M, W,
                       dxd, drop_p, drop_seed, tfk_seed_key(), dbias, (unsigned char*)mq, (unsigned char*)ms,
                       (unsigned char*)mqt, (unsigned char*)mst, part);
  else if (cpl <= 4)
    hipLaunchKernelGGL(ln_bwd_kernel<4>, grid, dim3(NT), sh, s, dy, x, gamma, mean, rstd, dres, dx, dgamma, dbeta, M, W,
                       dxd, drop_p, drop_seed, tfk_seed_key(), dbias, (unsigned char*)mq, (unsigned char*)ms,
                       (unsigned char*)mqt, (unsigned char*)mst, part);
  else return -3;
  if (part) {
    const int NS = dbias ? 3 : 2;
    // one group per <= 8 slabs (every load of a thread in flight at once), at least LN_PART_GROUPS
    const int groups = std::min(256, std::max(LN_PART_GROUPS, ((int)grid.x + 7) / 8));
    hipLaunchKernelGGL(ln_part_reduce_kernel, dim3((NS * W + NT - 1) / NT, groups), dim3(NT), 0, s, part,
                       (int)grid.x, NS, W, dgamma, dbeta, dbias);
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int tfk_embedding_fwd(const int* ids, const bf16* word, int V, const bf16* pos, int S, const int* tt, const bf16* type,
                      int T, bf16* out, long long ntok, int W, float scale, hipStream_t s) {
  hipLaunchKernelGGL(embed_fwd_kernel, dim3(grid_for(ntok * (W / 8), NT, 8192)), dim3(NT), 0, s, ids, word, V, pos, S,
                     tt, type, T, out, ntok, W, scale);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
// dpos (if given) is OVERWRITTEN for rows < S; dtype (T <= 4) is accumulated.
// scratch (optional): int32 [3 V + ntok] -> bucketed word-row gradient (no f32 atomics); null ->
// scattered atomics. dword rows must be 16-B aligned (W % 4 == 0) for the bucketed form.
int tfk_embedding_bwd(const int* ids, const bf16* dy, int V, float* dword, float* dpos, int S, const int* tt,
                      float* dtype, int T, long long ntok, int W, float scale, int* scratch, hipStream_t s) {
  if (dtype && T > 4) return -3;
  if (scratch && W % 8 == 0 && (((uintptr_t)dword) & 15) == 0) {
    int *cnt = scratch, *off = scratch + V, *cursor = scratch + 2 * (long long)V, *list = scratch + 3 * (long long)V;
    // counts zeroed by a KERNEL node, not hipMemsetAsync: a memset captured into a hipGraph whose
    // step also forks onto the RCCL comm stream was not ordered before the counting kernel on
    // replay (stale counts -> out-of-range bucket writes -> the round-4 illegal-address fault of the
    // captured transformer steps with collectives; profiles/perf_log_r5.md)
    hipLaunchKernelGGL(emb_zero_kernel, dim3((unsigned)min((V + NT - 1) / NT, 1024)), dim3(NT), 0, s, cnt, V);
    const unsigned g = (unsigned)grid_for(ntok, NT, 1024);
    hipLaunchKernelGGL(emb_count_kernel, dim3(g), dim3(NT), 0, s, ids, ntok, V, cnt);
    hipLaunchKernelGGL(emb_scan_kernel, dim3(1), dim3(1024), 0, s, cnt, V, off, cursor);
    hipLaunchKernelGGL(emb_bucket_kernel, dim3(g), dim3(NT), 0, s, ids, ntok, V, cursor, list);
    hipLaunchKernelGGL(emb_reduce_kernel, dim3((unsigned)V), dim3(NT), 0, s, off, cnt, list, dy, dword, W, scale, ntok);
  } else {
    hipLaunchKernelGGL(embed_bwd_kernel, dim3(grid_for(ntok * (W / 8), NT, 8192)), dim3(NT), 0, s, ids, dy, V, dword,
                       ntok, W, scale);
  }
  if (dpos)
    hipLaunchKernelGGL(embed_pos_bwd_kernel, dim3(grid_for((long long)S * (W / 8), NT, 4096)), dim3(NT), 0, s, dy, dpos,
                       S, (int)(ntok / S), W);
  if (dtype)
    hipLaunchKernelGGL(embed_type_bwd_kernel, dim3((W / 8 + NT - 1) / NT, 128), dim3(NT), 0, s, dy, tt, dtype, T, ntok,
                       W);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
}
// read and clear the bucketed-backward guard counter (host; synchronizes the device)
extern "C" int tfk_emb_guard_count() {
  int v = 0, z = 0;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_emb_guard), sizeof(int)) != hipSuccess) return -1;
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_emb_guard), &z, sizeof(int)) != hipSuccess) return -1;
  return v;
}
