// MX-fp8 (OCP e4m3 + e8m0 block scales) GEMM and quantizer for gfx950.
//
// gfx950 runs non-scaled fp8 MFMA at the bf16 rate; the 2x fp8 rate comes only from the
// block-scaled v_mfma_scale_f32_16x16x128_f8f6f4 (K = 128 per instruction, one e8m0 scale per
// 32 K-elements of each row, applied in hardware). So the fp8 path is MX: operands are quantized
// per (row, 32-wide K block) to e4m3 with a power-of-two scale chosen so the block max maps to
// <= 448 (no saturation), and the GEMM feeds the bytes and scales straight into the scaled MFMA.
//
// GEMM layout: A [M][K] and B [N][K] bytes (K-inner, K % 128 == 0), scales [rows][K/32]. A K-tile
// is 128 K-elements = 128 B per row: the same LDS image (128-B rows, XOR-swizzled 16-B chunks) and
// loader pattern as the bf16 engine's BK=64 tiles, plus the tile's 4 scale bytes per row staged in
// LDS. 256 threads (2x2 waves), 128x128 tiles, register-staged double buffering, one barrier per
// K-tile, the shared bf16 epilogue (bias/act/aux/dropout/residual; gemm_epilogue.h).
// MFMA operand map (measured with tools/mx_probe.py / tools/mx_diag.py, checked against a
// dequantized fp32 reference in tests/test_fp8_gpu.py): lane l holds row (l&15); its 32 operand
// bytes are K-elements 16g..16g+15 (bytes 0-15) and 64+16g..64+16g+15 (bytes 16-31), g = l>>4,
// i.e. 16-B chunks g and g+4 of the 128-B row. The scale operand of lane group g is the scale of
// K block g (K-elements 32g..32g+31), so the four scale bytes of a row go to groups 0..3 in order.
#include "common.h"
#include "gemm_params.h"
#include "gemm_epilogue.h"
#include "mx_common.h"

namespace tfk {
namespace {
typedef int i32x8 __attribute__((ext_vector_type(8)));
constexpr int NTF = 256;
constexpr int BKB = 128;  // K elements (bytes) per tile

__device__ __forceinline__ int kin_off8(int row, int kc) { return row * 128 + ((kc ^ ((row >> 1) & 7)) << 4); }

template <int ROWS>
struct Fp8Loader {
  static constexpr int NCH = ROWS * 8 / NTF;
  const unsigned char* tb;  // this thread's first chunk (k = 0)
  const unsigned char* sc;  // scale row of this thread (threads < ROWS), else null
  long long ld;
  int rows_valid;           // rows of this tile that exist
  __device__ __forceinline__ void init(const unsigned char* base, const unsigned char* scales, long long ld_, int row0,
                                       int lim, int sld, int sc_tid) {
    ld = ld_;
    rows_valid = lim - row0;
    tb = base + (long long)(row0 + (threadIdx.x >> 3)) * ld + (threadIdx.x & 7) * 16;
    sc = (sc_tid >= 0 && sc_tid < ROWS && row0 + sc_tid < lim) ? scales + (long long)(row0 + sc_tid) * sld : nullptr;
  }
  __device__ __forceinline__ void load(int kt, u32x4 (&r)[NCH], unsigned int& s) const {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int row = (threadIdx.x >> 3) + (NTF / 8) * i;
      r[i] = row < rows_valid ? *(const u32x4*)(tb + (long long)i * (NTF / 8) * ld + kt * BKB) : u32x4{0u, 0u, 0u, 0u};
    }
    s = sc ? *(const unsigned int*)(sc + kt * 4) : 0u;
  }
  __device__ __forceinline__ void store(char* lds, unsigned int* slds, int sc_tid, const u32x4 (&r)[NCH],
                                        unsigned int s) const {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int row = (threadIdx.x >> 3) + (NTF / 8) * i;
      *(u32x4*)(lds + kin_off8(row, threadIdx.x & 7)) = r[i];
    }
    if (sc_tid >= 0 && sc_tid < ROWS) slds[sc_tid] = s;
  }
};

__device__ __forceinline__ i32x8 frag8(const char* lds, int row, int g) {
  const u32x4 lo = *(const u32x4*)(lds + kin_off8(row, g));
  const u32x4 hi = *(const u32x4*)(lds + kin_off8(row, g + 4));
  i32x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

template <int BM, int BN, int EPI>
__global__ __launch_bounds__(NTF, 2) void mxfp8_gemm_kernel(GemmParams p) {
  constexpr int WM = 2, WN = 2, TM = BM / WM, TN = BN / WN, FM = TM / 16, FN = TN / 16;
  constexpr int A_BYTES = BM * BKB, B_BYTES = BN * BKB;
  constexpr int STAGE = A_BYTES + B_BYTES + (BM + BN) * 4;
  constexpr int MAIN = 2 * STAGE;
  constexpr int EPI_BYTES = epi_lds_bytes<BM, BN, WM>();
  __shared__ __attribute__((aligned(16))) char smem[MAIN > EPI_BYTES ? MAIN : EPI_BYTES];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = tile / p.tiles_n, tn = tile - tm * p.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int sld = p.K / 32;
  const int nkt = p.K / BKB;

  Fp8Loader<BM> la;
  Fp8Loader<BN> lb;
  la.init((const unsigned char*)p.A, (const unsigned char*)p.a_scale, p.lda, m0, p.M, sld, tid);
  lb.init((const unsigned char*)p.B, (const unsigned char*)p.b_scale, p.ldb, n0, p.N, sld, tid - BM);

  auto stage = [&](int b) { return smem + b * STAGE; };
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  u32x4 ra[Fp8Loader<BM>::NCH], rb[Fp8Loader<BN>::NCH];
  unsigned int sa = 0, sb = 0;
  if (nkt > 0) {
    la.load(0, ra, sa);
    lb.load(0, rb, sb);
    char* st = stage(0);
    la.store(st, (unsigned int*)(st + A_BYTES + B_BYTES), tid, ra, sa);
    lb.store(st + A_BYTES, (unsigned int*)(st + A_BYTES + B_BYTES) + BM, tid - BM, rb, sb);
  }
  __syncthreads();
  const int g = lane >> 4, li = lane & 15;
  for (int kt = 0; kt < nkt; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nkt;
    if (more) {
      la.load(kt + 1, ra, sa);
      lb.load(kt + 1, rb, sb);
    }
    const char* st = stage(cur);
    const unsigned int* ssa = (const unsigned int*)(st + A_BYTES + B_BYTES);
    const unsigned int* ssb = ssa + BM;
    i32x8 af[FM], bfr[FN];
    int sca[FM], scb[FN];
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int row = wm * TM + i * 16 + li;
      af[i] = frag8(st, row, g);
      sca[i] = (ssa[row] >> (8 * g)) & 0xff;
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int row = wn * TN + j * 16 + li;
      bfr[j] = frag8(st + A_BYTES, row, g);
      scb[j] = (ssb[row] >> (8 * g)) & 0xff;
    }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(bfr[j], af[i], acc[i][j], 0, 0, 0, scb[j], 0,
                                                                     sca[i]);
    if (more) {
      char* nx = stage(cur ^ 1);
      la.store(nx, (unsigned int*)(nx + A_BYTES + B_BYTES), tid, ra, sa);
      lb.store(nx + A_BYTES, (unsigned int*)(nx + A_BYTES + B_BYTES) + BM, tid - BM, rb, sb);
    }
    __syncthreads();
  }
  gemm_epilogue<BM, BN, NTF, WM, EPI>(p, acc, smem, m0, n0, 0);
}

// One MX block: 32 values -> 32 e4m3 bytes (w[0..7], little-endian in K order) + the e8m0 exponent.
// scale exponent e = ceil(log2(amax / 448)) so every |x| * 2^-e <= 448 (no saturation).
__device__ __forceinline__ int mx_block(const float (&v)[32], unsigned (&w)[8]) {
  float amax = 0.f;
#pragma unroll
  for (int e = 0; e < 32; ++e) amax = fmaxf(amax, fabsf(v[e]));
  int ex = amax > 0.f ? (int)ceilf(log2f(amax * (1.f / 448.f))) : -127;
  ex = ex < -127 ? -127 : (ex > 127 ? 127 : ex);
  const float inv = ldexpf(1.f, -ex);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    float a0 = fminf(fmaxf(v[4 * k] * inv, -448.f), 448.f), a1 = fminf(fmaxf(v[4 * k + 1] * inv, -448.f), 448.f);
    float a2 = fminf(fmaxf(v[4 * k + 2] * inv, -448.f), 448.f), a3 = fminf(fmaxf(v[4 * k + 3] * inv, -448.f), 448.f);
    int pk = __builtin_amdgcn_cvt_pk_fp8_f32(a0, a1, 0, false);
    pk = __builtin_amdgcn_cvt_pk_fp8_f32(a2, a3, pk, true);
    w[k] = (unsigned int)pk;
  }
  return ex;
}

// Both MX quantizations of x bf16 [R][C] in ONE read: row blocks (q_r [R][C], s_r [R][C/32], the
// forward / dgrad operand) and column blocks (q_c [C][R], s_c [C][R/32] = MX of x^T, the weight-
// gradient operand). Unit = a 128 x 128 tile staged in LDS (16-B lane-linear loads); 256 threads
// each quantize 2 row blocks and one column PAIR (2 column blocks, read as 32-bit LDS words).
// 128 x 128 makes every e4m3 store pattern full 128-B lines per tile: a row of q_r gets 4
// consecutive 32-B blocks, a row of q_c (a column of x) its 4 row groups (32-row tiles wrote each
// q_c line in 4 quarters from 4 blocks: 45% of the HBM floor in Transformer-big).
//
// v2: the block scale comes from the integer bf16 magnitudes (packed u16 max), the bytes from
// v_cvt_scalef32_pk_fp8_bf16 (two bf16 -> two e4m3, x / 2^e, RNE: exact against the reference, as
// 2^-e scaling of a bf16 is exact) -- no unpack / multiply / clamp per element. Resident blocks walk
// tiles (t += gridDim.x) with the next tile's 8 16-B loads in flight under this tile's quantize and
// stores. One launch can cover MANY tensors (a descriptor table: all weights of a model per step).
constexpr int QT = 128, QLD = QT + 8;
struct QDesc {
  const bf16* x;
  unsigned char *qr, *sr, *qc, *sc;
  int R, C;
  int t0, tcols;  // first tile of this tensor in the launch; column tiles
};
static_assert(sizeof(QDesc) == 56, "QDesc is packed as 7 int64 by ops/fp8.py");
__device__ __forceinline__ void qd_load(const QDesc& d, int lt, int t, u32x4 (&r)[8]) {
  const int r0 = (lt / d.tcols) * QT, c0 = (lt % d.tcols) * QT;
  const int rows = min(QT, d.R - r0), cols = min(QT, d.C - c0);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int idx = t + i * 256, row = idx >> 4, ch = (idx & 15) * 8;
    r[i] = (row < rows && ch < cols) ? *(const u32x4*)(d.x + (long long)(r0 + row) * d.C + c0 + ch)
                                     : u32x4{0u, 0u, 0u, 0u};
  }
}

template <bool TABLE>
__device__ __forceinline__ void qd_find(const QDesc* tab, int n, const QDesc& one, int t, QDesc& d) {
  if constexpr (!TABLE) {
    d = one;
  } else {
    int lo = 0, hi = n - 1;  // last entry with t0 <= t (block-uniform: scalar loads)
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (tab[mid].t0 <= t) lo = mid; else hi = mid - 1;
    }
    d = tab[lo];
  }
}

// The column blocks' e4m3 bytes and scales are staged in LDS ([128 columns][128 rows] bytes) and
// written as whole 128-B q_c lines (8 lanes per line, 8 lines per wave store): per-thread 32-B
// stores scattered over 128 rows ran the dual quantizer at ~4 TB/s against the row quantizer's
// 6.4 (profiles/mxq_bench_r3b.jsonl).
constexpr int QCL = QT + 16;
template <bool TABLE>
__global__ __launch_bounds__(256) void mx_quant_dual_kernel(QDesc one, const QDesc* __restrict__ tab, int n, int total) {
  __shared__ __attribute__((aligned(16))) bf16 tile[QT][QLD];
  __shared__ __attribute__((aligned(16))) unsigned char qcl[QT][QCL];
  __shared__ __attribute__((aligned(16))) unsigned char scl[QT][4];
  const int t = threadIdx.x;
  int ti = blockIdx.x;
  if (ti >= total) return;
  QDesc d;
  qd_find<TABLE>(tab, n, one, ti, d);
  u32x4 rg[8];
  qd_load(d, ti - d.t0, t, rg);
  while (true) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int idx = t + i * 256;
      *(u32x4*)&tile[idx >> 4][(idx & 15) * 8] = rg[i];
    }
    __syncthreads();
    const int tn = ti + gridDim.x;  // block-uniform
    QDesc dn;
    if (tn < total) {
      qd_find<TABLE>(tab, n, one, tn, dn);
      qd_load(dn, tn - dn.t0, t, rg);  // in flight under this tile's quantize + stores
    }
    const int lt = ti - d.t0, r0 = (lt / d.tcols) * QT, c0 = (lt % d.tcols) * QT;
    const int rows = min(QT, d.R - r0), cols = min(QT, d.C - c0);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int pr = t + k * 256, row = pr >> 2, blk = pr & 3;
      if (row < rows && blk * 32 < cols) {
        unsigned p[16];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const u32x4 h = *(const u32x4*)&tile[row][blk * 32 + q * 8];
          p[4 * q] = h[0]; p[4 * q + 1] = h[1]; p[4 * q + 2] = h[2]; p[4 * q + 3] = h[3];
        }
        unsigned w[8];
        const int ex = mx_block_pk(p, w);
        const int c = c0 + blk * 32;
        unsigned char* dst = d.qr + (long long)(r0 + row) * d.C + c;
        *(u32x4*)dst = u32x4{w[0], w[1], w[2], w[3]};
        *(u32x4*)(dst + 16) = u32x4{w[4], w[5], w[6], w[7]};
        d.sr[(long long)(r0 + row) * (d.C / 32) + c / 32] = (unsigned char)(ex + 127);
      }
    }
    {
      // column pair (2cp, 2cp+1), rows rgp*32 .. +32: one 32-bit LDS word per row holds both
      const int cp = t & 63, rgp = t >> 6, col = 2 * cp;
      if (col < cols && rgp * 32 < rows) {
        unsigned lo[16], hi[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const unsigned a = *(const unsigned*)&tile[rgp * 32 + 2 * r][col];
          const unsigned b = *(const unsigned*)&tile[rgp * 32 + 2 * r + 1][col];
          lo[r] = __builtin_amdgcn_perm(b, a, 0x05040100u);  // (a.lo, b.lo): column col, rows 2r, 2r+1
          hi[r] = __builtin_amdgcn_perm(b, a, 0x07060302u);  // (a.hi, b.hi): column col + 1
        }
        unsigned w[8];
        int ex = mx_block_pk(lo, w);
        *(u32x4*)&qcl[col][rgp * 32] = u32x4{w[0], w[1], w[2], w[3]};
        *(u32x4*)&qcl[col][rgp * 32 + 16] = u32x4{w[4], w[5], w[6], w[7]};
        scl[col][rgp] = (unsigned char)(ex + 127);
        ex = mx_block_pk(hi, w);
        *(u32x4*)&qcl[col + 1][rgp * 32] = u32x4{w[0], w[1], w[2], w[3]};
        *(u32x4*)&qcl[col + 1][rgp * 32 + 16] = u32x4{w[4], w[5], w[6], w[7]};
        scl[col + 1][rgp] = (unsigned char)(ex + 127);
      }
    }
    __syncthreads();  // column bytes staged; every read of the bf16 tile retired
    {
      const long long R = d.R;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int idx = t + i * 256, c = idx >> 3, ch = (idx & 7) * 16;
        if (c < cols && ch < rows) *(u32x4*)(d.qc + (long long)(c0 + c) * R + r0 + ch) = *(const u32x4*)&qcl[c][ch];
      }
      if (t < cols) {
        unsigned char* sdst = d.sc + (long long)(c0 + t) * (R / 32) + r0 / 32;
        if (rows == QT && ((R / 32) & 3) == 0) {
          *(unsigned*)sdst = *(const unsigned*)&scl[t][0];
        } else {
          for (int g = 0; g * 32 < rows; ++g) sdst[g] = scl[t][g];
        }
      }
    }
    if (tn >= total) break;
    ti = tn;
    d = dn;
  }
}

// x bf16 [rows][K] -> q e4m3 [rows][K] + s e8m0 [rows][K/32]; one thread per 32-element block.
__global__ void mx_quant_kernel(const bf16* __restrict__ x, unsigned char* __restrict__ q,
                                unsigned char* __restrict__ s, long long nblocks) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < nblocks; i += (long long)gridDim.x * 256) {
    const bf16* src = x + i * 32;
    float v[32];
    float amax = 0.f;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      bf16x8 t = *(const bf16x8*)(src + c * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) { v[c * 8 + e] = bf2f(t[e]); amax = fmaxf(amax, fabsf(v[c * 8 + e])); }
    }
    int ex = amax > 0.f ? (int)ceilf(log2f(amax * (1.f / 448.f))) : -127;
    ex = ex < -127 ? -127 : (ex > 127 ? 127 : ex);
    const float inv = ldexpf(1.f, -ex);
    unsigned int w[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float a0 = fminf(fmaxf(v[4 * k] * inv, -448.f), 448.f), a1 = fminf(fmaxf(v[4 * k + 1] * inv, -448.f), 448.f);
      float a2 = fminf(fmaxf(v[4 * k + 2] * inv, -448.f), 448.f), a3 = fminf(fmaxf(v[4 * k + 3] * inv, -448.f), 448.f);
      int pk = __builtin_amdgcn_cvt_pk_fp8_f32(a0, a1, 0, false);
      pk = __builtin_amdgcn_cvt_pk_fp8_f32(a2, a3, pk, true);
      w[k] = (unsigned int)pk;
    }
    *(u32x4*)(q + i * 32) = u32x4{w[0], w[1], w[2], w[3]};
    *(u32x4*)(q + i * 32 + 16) = u32x4{w[4], w[5], w[6], w[7]};
    s[i] = (unsigned char)(ex + 127);
  }
}
// Transposing quantizer for the backward GEMMs: x bf16 [R][C] (row-major) -> q e4m3 [C][R] with
// s e8m0 [C][R/32], i.e. the MX blocks run along R (the reduction dimension of dgrad's W^T and of
// wgrad's dY^T / X^T). Block = 256 threads = a 32-row x 256-column tile staged through LDS with
// 16-B loads; thread t then owns column t: amax over its 32 values (LDS reads of one row by a wave
// are 128 contiguous bytes: conflict-free), one exponent, 32 e4m3 bytes written as two 16-B stores.
// R % 32 == 0 (host-checked); ragged C is masked.
__global__ void mx_quant_t_kernel(const bf16* __restrict__ x, unsigned char* __restrict__ q,
                                  unsigned char* __restrict__ s, int R, int C) {
  __shared__ bf16 tile[32][256 + 8];
  const int r0 = blockIdx.y * 32, c0 = blockIdx.x * 256, t = threadIdx.x;
  const bool vec = (C & 7) == 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {  // 32 rows x 32 chunks of 8 columns = 1024 chunks / 256 threads
    const int idx = t + i * 256, row = idx >> 5, ch = (idx & 31) * 8;
    const int c = c0 + ch;
    const bf16* src = x + (long long)(r0 + row) * C + c;
    if (vec && c + 8 <= C) {
      *(bf16x8*)&tile[row][ch] = *(const bf16x8*)src;
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) tile[row][ch + e] = c + e < C ? src[e] : f2bf(0.f);
    }
  }
  __syncthreads();
  const int c = c0 + t;
  if (c >= C) return;
  float v[32];
  float amax = 0.f;
#pragma unroll
  for (int r = 0; r < 32; ++r) { v[r] = bf2f(tile[r][t]); amax = fmaxf(amax, fabsf(v[r])); }
  int ex = amax > 0.f ? (int)ceilf(log2f(amax * (1.f / 448.f))) : -127;
  ex = ex < -127 ? -127 : (ex > 127 ? 127 : ex);
  const float inv = ldexpf(1.f, -ex);
  unsigned int w[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    float a0 = fminf(fmaxf(v[4 * k] * inv, -448.f), 448.f), a1 = fminf(fmaxf(v[4 * k + 1] * inv, -448.f), 448.f);
    float a2 = fminf(fmaxf(v[4 * k + 2] * inv, -448.f), 448.f), a3 = fminf(fmaxf(v[4 * k + 3] * inv, -448.f), 448.f);
    int pk = __builtin_amdgcn_cvt_pk_fp8_f32(a0, a1, 0, false);
    pk = __builtin_amdgcn_cvt_pk_fp8_f32(a2, a3, pk, true);
    w[k] = (unsigned int)pk;
  }
  unsigned char* dst = q + (long long)c * R + r0;
  *(u32x4*)dst = u32x4{w[0], w[1], w[2], w[3]};
  *(u32x4*)(dst + 16) = u32x4{w[4], w[5], w[6], w[7]};
  s[(long long)c * (R / 32) + blockIdx.y] = (unsigned char)(ex + 127);
}

// One-wave self-test of the scaled MFMA operand maps: X/Y are [64 lanes][8] words, scales one per
// lane, D [64 lanes][4] (lane-major) = mfma_scale(X, Y) (tests/test_fp8_gpu.py probes the layout).
__global__ void mx_probe_kernel(const int* X, const int* Y, const int* sx, const int* sy, float* D) {
  const int l = threadIdx.x;
  i32x8 x, y;
#pragma unroll
  for (int e = 0; e < 8; ++e) { x[e] = X[l * 8 + e]; y[e] = Y[l * 8 + e]; }
  f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(x, y, acc, 0, 0, 0, sx[l], 0, sy[l]);
#pragma unroll
  for (int r = 0; r < 4; ++r) D[l * 4 + r] = acc[r];
}
}  // namespace
}  // namespace tfk

using namespace tfk;

extern "C" {
int tfk_mx_probe(const int* X, const int* Y, const int* sx, const int* sy, float* D, hipStream_t st) {
  hipLaunchKernelGGL(mx_probe_kernel, dim3(1), dim3(64), 0, st, X, Y, sx, sy, D);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int tfk_mx_quant_t(const void* x, void* q, void* s, int R, int C, hipStream_t st) {
  if (R % 32 || R <= 0 || C <= 0) return -1;
  dim3 grid((unsigned)((C + 255) / 256), (unsigned)(R / 32));
  hipLaunchKernelGGL(mx_quant_t_kernel, grid, dim3(256), 0, st, (const bf16*)x, (unsigned char*)q, (unsigned char*)s, R, C);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
// resident dual-quantizer blocks: 4 per CU fit the 34 KiB tile (TFK_MXQ_GRID overrides, for A/B)
static int mxq_grid(int total) {
  static int g = -1;
  if (g < 0) {
    const char* e = getenv("TFK_MXQ_GRID");
    g = e ? atoi(e) : 1024;
    if (g < 1) g = 1024;
  }
  return total < g ? total : g;
}
int tfk_mx_quant_dual(const void* x, void* qr, void* sr, void* qc, void* sc, int R, int C, hipStream_t st) {
  if (R % 32 || C % 32 || R <= 0 || C <= 0) return -1;
  QDesc d{(const bf16*)x, (unsigned char*)qr, (unsigned char*)sr, (unsigned char*)qc, (unsigned char*)sc, R, C, 0,
          (C + QT - 1) / QT};
  const int total = d.tcols * ((R + QT - 1) / QT);
  hipLaunchKernelGGL(mx_quant_dual_kernel<false>, dim3((unsigned)mxq_grid(total)), dim3(256), 0, st, d,
                     (const QDesc*)nullptr, 1, total);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
// Many tensors in one launch: tab = n device-resident QDesc (t0 ascending, each R, C % 32 == 0).
int tfk_mx_quant_dual_group(const void* tab, int n, int total, hipStream_t st) {
  if (n <= 0 || total <= 0) return -1;
  QDesc none{};
  hipLaunchKernelGGL(mx_quant_dual_kernel<true>, dim3((unsigned)mxq_grid(total)), dim3(256), 0, st, none,
                     (const QDesc*)tab, n, total);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int tfk_mx_quant(const void* x, void* q, void* s, long long nblocks, hipStream_t st) {
  long long g = (nblocks + 255) / 256;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(mx_quant_kernel, dim3((unsigned)g), dim3(256), 0, st, (const bf16*)x, (unsigned char*)q,
                     (unsigned char*)s, nblocks);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
// C[M][N] = epilogue(A q[M][K] x B q[N][K]^T), scales in p.a_scale / p.b_scale.
// ext: 0 bf16 (bias/act/resid), 1 bf16 EXT (aux, dropout, activation backward), 2 f32 (alpha/beta:
// weight gradients accumulate into the f32 arena), 3 EXT + MX-fp8 copies of the output (p.mx_*).
extern "C" int tfk_g4_fp8_launch(const GemmParams& p, int epi, int splits, hipStream_t stream);
// 1 = g4 LDS-DMA engine (default; 256x256 16-wave tiles measured 1.4-1.7x the bf16 g4 GEMM,
// profiles/fp8_engine_r3a.jsonl), 0 = the register-staged kernel below (TFK_FP8_ENGINE=reg).
static int g_fp8_engine = -1;
extern "C" void tfk_fp8_set_engine(int e) { g_fp8_engine = e; }
// splits: split-K count of the f32 (weight-gradient) output, slab z at C + z * p.split_stride (the
// register engine below runs unsplit: only the g4 engine takes splits > 1).
int tfk_gemm_mxfp8(GemmParams p, int ext, int splits, hipStream_t st) {
  if (g_fp8_engine < 0) {
    const char* e = getenv("TFK_FP8_ENGINE");
    g_fp8_engine = (e && e[0] == 'r') ? 0 : 1;
  }
  if (g_fp8_engine == 1) {
    const int r = tfk_g4_fp8_launch(p, ext == 3 ? EPI_BF16_EXT_MX : ext == 2 ? EPI_F32 : (ext ? EPI_BF16_EXT : EPI_BF16),
                                    splits, st);
    if (r != -1 || ext == 3) return r;
  }
  if (splits > 1 || ext == 3) return -1;  // MX-output epilogue: g4 engine only
  const int BM = 128, BN = 128;
  p.tiles_n = (p.N + BN - 1) / BN;
  if (p.stats_shards < 1) p.stats_shards = 1;
  dim3 grid(((p.M + BM - 1) / BM) * p.tiles_n, 1, 1);
  if (ext == 2)
    hipLaunchKernelGGL((mxfp8_gemm_kernel<128, 128, EPI_F32>), grid, dim3(NTF), 0, st, p);
  else if (ext)
    hipLaunchKernelGGL((mxfp8_gemm_kernel<128, 128, EPI_BF16_EXT>), grid, dim3(NTF), 0, st, p);
  else
    hipLaunchKernelGGL((mxfp8_gemm_kernel<128, 128, EPI_BF16>), grid, dim3(NTF), 0, st, p);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
}
