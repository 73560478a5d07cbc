// tfk MFMA implicit-GEMM engine for gfx950 (CDNA4).
//
// One templated kernel computes C[M,N] = epilogue( sum_k A(m,k) * B(n,k) ) where each operand is
// read either "K-inner" (row-major [rows][K], LDS image read with ds_read_b128) or "K-outer"
// ([K][rows], LDS image read with the gfx950 hardware-transpose ds_read_b64_tr_b16), optionally
// through an NHWC convolution gather:
//   A_CONV_FWD   : A(m=(n,p,q), k=(r,s,c))  = X[n, p*sh-ph+r*dh, q*sw-pw+s*dw, c]        (conv fwd)
//   A_CONV_DGRAD : A(m=(n,h,w), k=(r,s,co)) = dY[n, (h+ph-r*dh)/sh, (w+pw-s*dw)/sw, co]  (conv dgrad)
//   B_CONV_WGRAD : B(n=(r,s,c), k=(n,p,q))  = X[n, p*sh-ph+r*dh, q*sw-pw+s*dw, c]        (conv wgrad)
// Zero padding comes for free from predicated (zero-filled) register-staged loads.
//
// Structure (cdna_hip_programming.md §5): 256 threads = 4 waves (2x2), BK=64, two LDS buffers,
// one barrier per K-tile, global loads for tile k+1 issued before the MFMAs of tile k and written
// to LDS after them (T14 issue-early/write-late). v_mfma_f32_16x16x32_bf16, f32 accumulate.
// LDS images are XOR-swizzled so both the b128 row reads and the tr_b16 column reads are
// bank-conflict-free (derivation in docs/KERNELS.md). Block ids are XCD-remapped (T1).
// Epilogues: bf16 (alpha, bias, relu/gelu, residual add, fused BatchNorm batch-statistics
// partial sums via sharded atomics) staged through LDS for 16-B coalesced stores, or f32
// (split-K slabs / beta-accumulate) stored straight from the accumulators.
#include "common.h"
#include "gemm_params.h"

namespace tfk {

enum AMode { A_KIN = 0, A_KOUT = 1, A_CONV_FWD = 2, A_CONV_DGRAD = 3 };
enum BMode { B_KIN = 0, B_KOUT = 1, B_CONV_WGRAD = 2 };
// BNR: + fused BN-backward reduction; EXT: + aux (pre-activation) store, activation-backward
// multiplier and dropout. Separate instantiations keep the common epilogue small enough to unroll
// fully (a rolled epilogue indexes the accumulators dynamically -> they go to scratch).
enum EpiMode { EPI_BF16 = 0, EPI_F32 = 1, EPI_BF16_BNR = 2, EPI_BF16_EXT = 3 };

// GemmParams lives in gemm_params.h (shared with the host bindings).


constexpr int BK = 64;
// Threads per block: 8 waves (2x4 wave grid, 128x64 per wave) for the 256x256 tile, else 4 waves
// (2x2). The big tile halves the LDS fragment reads per MFMA (12 ds_read per 32 MFMA vs 8 per 16)
// and the global->LDS bytes per FLOP; 128 KiB of double-buffered LDS -> 1 block (8 waves) per CU.
template <int BM, int BN>
constexpr int threads_for() { return (BM >= 256 && BN >= 256) ? 512 : 256; }

template <int ROWS>
__device__ __forceinline__ int swz_kout(int k) {
  if constexpr (ROWS >= 128) return 2 * ((k & 3) | (((k >> 3) & 1) << 2));
  else return 2 * (((k >> 1) & 1) | (((k >> 3) & 1) << 1));
}

// Byte offset of chunk (row, kc) in a K-inner [ROWS][64] image (128-B rows).
__device__ __forceinline__ int kin_off(int row, int kc) { return row * 128 + ((kc ^ ((row >> 1) & 7)) << 4); }
// Byte offset of chunk (krow, rc) in a K-outer [64][ROWS] image.
template <int ROWS>
__device__ __forceinline__ int kout_off(int krow, int rc) { return krow * (ROWS * 2) + ((rc ^ swz_kout<ROWS>(krow)) << 4); }

// Predicated scalar load of up to 8 consecutive bf16 (ragged tails / unaligned leading dims).
// Built from constant-index register words: a union/array indexed by a loop variable would be
// placed in scratch memory and drag the whole register-staged tile through it.
__device__ __forceinline__ u32x4 load_partial(const bf16* src, int valid, int stride) {
  const unsigned short* s = (const unsigned short*)src;
  unsigned int w[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const unsigned int lo = (2 * q < valid) ? (unsigned int)s[(2 * q) * stride] : 0u;
    const unsigned int hi = (2 * q + 1 < valid) ? (unsigned int)s[(2 * q + 1) * stride] : 0u;
    w[q] = lo | (hi << 16);
  }
  return u32x4{w[0], w[1], w[2], w[3]};
}

// Per-operand loader state. ROWS = tile rows of this operand (BM for A, BN for B).
template <int ROWS, int MODE, bool IS_A, int NT>
struct Loader {
  static constexpr bool KOUT = IS_A ? (MODE == A_KOUT) : (MODE == B_KOUT || MODE == B_CONV_WGRAD);
  static constexpr int NCH = ROWS * 8 / NT;  // 16-B chunks per thread per K-tile
  static constexpr int CPR = ROWS / 8;       // chunks per k-row (K-outer)
  static_assert(NT % CPR == 0 || !KOUT, "K-outer loader needs NT % (ROWS/8) == 0");
  const bf16* base;
  long long ld;
  int lim_rows, K;
  // dense fast path: block-uniform "every row of this tile is in range and 16-B aligned"
  bool full;
  const bf16* tbase;  // this thread's first chunk address (k = 0)
  // conv state
  long long rbase[NCH];
  int hb[NCH], wb[NCH];
  bool rv[NCH];
  int cr, cs, cc;  // (r, s, c) of this thread's chunk column for the current K-tile
  int fr, fs, fc;  // wgrad: fixed (r, s, c) of this thread's column chunk
  bool fvalid;

  __device__ __forceinline__ int chunk_row(int i) const {
    if constexpr (KOUT) return (threadIdx.x / CPR) + (NT / CPR) * i;
    else return (threadIdx.x >> 3) + (NT / 8) * i;
  }
  __device__ __forceinline__ int chunk_col() const {
    if constexpr (KOUT) return threadIdx.x % CPR;
    else return threadIdx.x & 7;
  }

  __device__ __forceinline__ void init(const GemmParams& p, const bf16* b, long long ld_, int row0, int rows, int kt0) {
    base = b; ld = ld_; lim_rows = rows; K = p.K;
    if constexpr (MODE == 0 || MODE == 1) {
      full = (row0 + ROWS <= rows) && ((ld & 7) == 0);
      if constexpr (!KOUT) tbase = b + (long long)(row0 + chunk_row(0)) * ld + chunk_col() * 8;
      else tbase = b + (long long)chunk_row(0) * ld + row0 + chunk_col() * 8;
    }
    if constexpr (IS_A && MODE == A_CONV_FWD) {
      const int PQ = p.P * p.Q;
#pragma unroll
      for (int i = 0; i < NCH; ++i) {
        int m = row0 + chunk_row(i);
        rv[i] = m < rows;
        int mm = rv[i] ? m : 0;
        int n = mm / PQ, rem = mm - n * PQ, pp = rem / p.Q, qq = rem - pp * p.Q;
        hb[i] = pp * p.sh - p.ph; wb[i] = qq * p.sw - p.pw;
        rbase[i] = (long long)n * p.H * p.W * p.Cin;
      }
      int k = kt0 * BK + chunk_col() * 8;
      cc = k % p.Cin; int rs = k / p.Cin; cr = rs / p.S; cs = rs - cr * p.S;
    } else if constexpr (IS_A && MODE == A_CONV_DGRAD) {
      const int HW = p.H * p.W;
#pragma unroll
      for (int i = 0; i < NCH; ++i) {
        int m = row0 + chunk_row(i);
        rv[i] = m < rows;
        int mm = rv[i] ? m : 0;
        int n = mm / HW, rem = mm - n * HW, h = rem / p.W, w = rem - h * p.W;
        hb[i] = h + p.ph; wb[i] = w + p.pw;
        rbase[i] = (long long)n * p.P * p.Q * p.Cout;
      }
      int k = kt0 * BK + chunk_col() * 8;
      cc = k % p.Cout; int rs = k / p.Cout; cr = rs / p.S; cs = rs - cr * p.S;
    } else if constexpr (!IS_A && MODE == B_CONV_WGRAD) {
      int col = row0 + chunk_col() * 8;
      fvalid = col < rows;
      int cl = fvalid ? col : 0;
      fc = cl % p.Cin; int rs = cl / p.Cin; fr = rs / p.S; fs = rs - fr * p.S;
    }
  }

  // Advance conv (r,s,c) tracking by one K-tile.
  __device__ __forceinline__ void advance(int C) {
    cc += BK;
    while (cc >= C) { cc -= C; if (++cs == S_) { cs = 0; ++cr; } }
  }
  int S_;

  __device__ __forceinline__ void load(const GemmParams& p, int kt, int row0, u32x4 (&regs)[NCH]) {
    const u32x4 zero = {0u, 0u, 0u, 0u};
    if constexpr (MODE == 0 || MODE == 1) {
      // interior tile, full K-tile: unpredicated 16-B loads, scalar strides (one uniform branch)
      if (full && (kt + 1) * BK <= K) {
        if constexpr (!KOUT) {
          const bf16* src = tbase + kt * BK;
#pragma unroll
          for (int i = 0; i < NCH; ++i) regs[i] = *(const u32x4*)(src + (long long)i * (NT / 8) * ld);
        } else {
          const bf16* src = tbase + (long long)kt * BK * ld;
#pragma unroll
          for (int i = 0; i < NCH; ++i) regs[i] = *(const u32x4*)(src + (long long)i * (NT / CPR) * ld);
        }
        return;
      }
    }
    if constexpr (MODE == 0 /*KIN dense (A_KIN==B_KIN==0)*/) {
      const int k = kt * BK + chunk_col() * 8;
      const bool vec = (ld & 7) == 0;
#pragma unroll
      for (int i = 0; i < NCH; ++i) {
        int r = row0 + chunk_row(i);
        bool ok = (r < lim_rows) && (k < K);
        const bf16* src = base + (long long)r * ld + k;
        if (ok && vec && k + 8 <= K) regs[i] = *(const u32x4*)src;
        else regs[i] = ok ? load_partial(src, K - k, 1) : zero;
      }
    } else if constexpr (MODE == 1 /*KOUT dense*/) {
      const int col = row0 + chunk_col() * 8;
      const bool vec = (ld & 7) == 0;
#pragma unroll
      for (int i = 0; i < NCH; ++i) {
        int k = kt * BK + chunk_row(i);
        bool ok = (k < K) && (col < lim_rows);
        const bf16* src = base + (long long)k * ld + col;
        if (ok && vec && col + 8 <= lim_rows) regs[i] = *(const u32x4*)src;
        else regs[i] = ok ? load_partial(src, lim_rows - col, 1) : zero;
      }
    } else if constexpr (IS_A && MODE == A_CONV_FWD) {
      const bool kok = cr < p.R;
      const long long koff = ((long long)(cr * p.dh) * p.W + cs * p.dw) * p.Cin + cc;
#pragma unroll
      for (int i = 0; i < NCH; ++i) {
        int h = hb[i] + cr * p.dh, w = wb[i] + cs * p.dw;
        bool ok = kok && rv[i] && (unsigned)h < (unsigned)p.H && (unsigned)w < (unsigned)p.W;
        long long off = rbase[i] + ((long long)hb[i] * p.W + wb[i]) * p.Cin + koff;
        regs[i] = ok ? *(const u32x4*)(base + off) : zero;
      }
    } else if constexpr (IS_A && MODE == A_CONV_DGRAD) {
      const bool kok = cr < p.R;
#pragma unroll
      for (int i = 0; i < NCH; ++i) {
        int th = hb[i] - cr * p.dh, tw = wb[i] - cs * p.dw;
        bool ok = kok && rv[i] && th >= 0 && tw >= 0;
        int pp, qq;
        if (p.sh == 1) { pp = th; } else { pp = th / p.sh; ok = ok && (pp * p.sh == th); }
        if (p.sw == 1) { qq = tw; } else { qq = tw / p.sw; ok = ok && (qq * p.sw == tw); }
        ok = ok && pp < p.P && qq < p.Q;
        long long off = rbase[i] + ((long long)pp * p.Q + qq) * p.Cout + cc;
        regs[i] = ok ? *(const u32x4*)(base + off) : zero;
      }
    } else if constexpr (!IS_A && MODE == B_CONV_WGRAD) {
      const int PQ = p.P * p.Q;
#pragma unroll
      for (int i = 0; i < NCH; ++i) {
        int k = kt * BK + chunk_row(i);
        bool ok = fvalid && k < K;
        int kk = ok ? k : 0;
        int n = kk / PQ, rem = kk - n * PQ, pp = rem / p.Q, qq = rem - pp * p.Q;
        int h = pp * p.sh - p.ph + fr * p.dh, w = qq * p.sw - p.pw + fs * p.dw;
        ok = ok && (unsigned)h < (unsigned)p.H && (unsigned)w < (unsigned)p.W;
        long long off = (((long long)n * p.H + h) * p.W + w) * p.Cin + fc;
        regs[i] = ok ? *(const u32x4*)(base + off) : zero;
      }
    }
  }

  __device__ __forceinline__ void store_lds(char* lds, const u32x4 (&regs)[NCH]) const {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      int off;
      if constexpr (KOUT) off = kout_off<ROWS>(chunk_row(i), chunk_col());
      else off = kin_off(chunk_row(i), chunk_col());
      *(u32x4*)(lds + off) = regs[i];
    }
  }
};

// Read one 16x(k=32) MFMA operand fragment for rows [rb, rb+16) and K-half kk from an LDS image.
template <int ROWS, bool KOUT>
__device__ __forceinline__ bf16x8 read_frag(const char* lds, int rb, int kk) {
  const int l = threadIdx.x & 63;
  if constexpr (!KOUT) {
    const int row = rb + (l & 15);
    return *(const bf16x8*)(lds + kin_off(row, kk * 4 + (l >> 4)));
  } else {
    const int g = l >> 4, i = l & 15, q = i >> 2, pc = i & 3;
    const int k0 = kk * 32 + 8 * g + q, k1 = k0 + 4;
    const int ch = (rb >> 3) + (pc >> 1);
    const int o0 = k0 * (ROWS * 2) + ((ch ^ swz_kout<ROWS>(k0)) << 4) + (pc & 1) * 8;
    const int o1 = k1 * (ROWS * 2) + ((ch ^ swz_kout<ROWS>(k1)) << 4) + (pc & 1) * 8;
    bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((LDS_AS bf16x4*)(lds + o0));
    bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((LDS_AS bf16x4*)(lds + o1));
    bf16x8 r;
    r.lo = lo; r.hi = hi;
    return r;
  }
}

template <int BM, int BN, int AM, int BMD, int EPI>
__global__ __launch_bounds__((threads_for<BM, BN>()), (threads_for<BM, BN>() == 512 ? 1 : 2)) void gemm_kernel(GemmParams p) {
  constexpr int NT = threads_for<BM, BN>();
  constexpr int NW = NT / 64;                    // waves
  constexpr int WM = 2, WN = NW / WM;            // wave grid
  constexpr int TM = BM / WM, TN = BN / WN;      // wave tile
  constexpr int FM = TM / 16, FN = TN / 16;      // 16x16 fragments per wave
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  constexpr bool A_KOUT_ = (AM == A_KOUT);
  constexpr bool B_KOUT_ = (BMD == B_KOUT || BMD == B_CONV_WGRAD);
  constexpr int MAIN_BYTES = 2 * (A_BYTES + B_BYTES);
  constexpr int EPI_BYTES = (EPI == EPI_F32) ? 0 : BM * (BN + 8) * 2;
  __shared__ __attribute__((aligned(16))) char smem[MAIN_BYTES > EPI_BYTES ? MAIN_BYTES : EPI_BYTES];
  char* As = smem;
  char* Bs = smem + 2 * A_BYTES;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = tile / p.tiles_n, tn = tile - tm * p.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int bz = blockIdx.y;
  const bf16* Ab = (const bf16*)p.A + bz * p.sA;
  const bf16* Bb = (const bf16*)p.B + bz * p.sB;

  const int nkt = (p.K + BK - 1) / BK;
  const int kt0 = blockIdx.z * p.kt_per_split;
  const int kt1 = min(nkt, kt0 + p.kt_per_split);

  Loader<BM, AM, true, NT> la;
  Loader<BN, BMD, false, NT> lb;
  la.S_ = p.S; lb.S_ = p.S;
  la.init(p, Ab, p.lda, m0, p.M, kt0);
  lb.init(p, Bb, p.ldb, n0, p.N, kt0);

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  u32x4 ra[Loader<BM, AM, true, NT>::NCH], rb[Loader<BN, BMD, false, NT>::NCH];
  if (kt0 < kt1) {
    la.load(p, kt0, m0, ra);
    lb.load(p, kt0, n0, rb);
    la.store_lds(As, ra);
    lb.store_lds(Bs, rb);
  }
  __syncthreads();

  for (int kt = kt0; kt < kt1; ++kt) {
    const int cur = (kt - kt0) & 1;
    const bool more = kt + 1 < kt1;
    if (more) {
      if constexpr (AM == A_CONV_FWD) la.advance(p.Cin);
      if constexpr (AM == A_CONV_DGRAD) la.advance(p.Cout);
      la.load(p, kt + 1, m0, ra);
      lb.load(p, kt + 1, n0, rb);
    }
    const char* Ac = As + cur * A_BYTES;
    const char* Bc = Bs + cur * B_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = read_frag<BM, A_KOUT_>(Ac, wm * TM + i * 16, kk);
#pragma unroll
      for (int j = 0; j < FN; ++j) bfr[j] = read_frag<BN, B_KOUT_>(Bc, wn * TN + j * 16, kk);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    }
    if (more) {
      la.store_lds(As + (cur ^ 1) * A_BYTES, ra);
      lb.store_lds(Bs + (cur ^ 1) * B_BYTES, rb);
    }
    __syncthreads();
  }

  // Accumulator (i,j) of this lane holds C[m][n..n+3] with
  //   m = m0 + wm*TM + i*16 + (lane&15),  n = n0 + wn*TN + j*16 + (lane>>4)*4.
  const int ml = lane & 15, nl = (lane >> 4) * 4;
  if constexpr (EPI == EPI_F32) {
    float* C = (float*)p.C + bz * p.sC + (long long)blockIdx.z * p.split_stride;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int m = m0 + wm * TM + i * 16 + ml;
      if (m >= p.M) continue;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = n0 + wn * TN + j * 16 + nl;
        float* dst = C + (long long)m * p.ldc + n;
        f32x4 v = acc[i][j] * p.alpha;
        if (n + 3 < p.N && (p.ldc & 3) == 0) {
          if (p.beta != 0.f) v += p.beta * *(f32x4*)dst;
          *(f32x4*)dst = v;
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (n + r < p.N) dst[r] = v[r] + (p.beta != 0.f ? p.beta * dst[r] : 0.f);
        }
      }
    }
  } else {
    constexpr int LDC_S = BN + 8;  // padded bf16 row stride of the LDS C tile
    bf16* Cs = (bf16*)smem;
    float csum[FN][4], csq[FN][4];
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) { csum[j][r] = 0.f; csq[j][r] = 0.f; }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int nloc = wn * TN + j * 16 + nl;
      float bv[4] = {0.f, 0.f, 0.f, 0.f};
      if (p.bias) {
#pragma unroll
        for (int r = 0; r < 4; ++r) bv[r] = (n0 + nloc + r < p.N) ? p.bias[n0 + nloc + r] : 0.f;
      }
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int mloc = wm * TM + i * 16 + ml;
        bf16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = acc[i][j][r] * p.alpha + bv[r];
          if constexpr (EPI != EPI_BF16_EXT) v = act_apply(v, p.act);  // EXT: in the store pass
          csum[j][r] += v;
          csq[j][r] += v * v;
          o[r] = f2bf(v);
        }
        *(bf16x4*)(Cs + mloc * LDC_S + nloc) = o;
      }
    }
    if (p.stats) {
      // rows >= M were zero-filled -> contribute 0 (no bias in conv use).
      float* st = p.stats + (long long)(blockIdx.x % p.stats_shards) * 2 * p.N;
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float s = csum[j][r], q = csq[j][r];
#pragma unroll
          for (int o = 1; o < 16; o <<= 1) { s += __shfl_xor(s, o, 64); q += __shfl_xor(q, o, 64); }
          const int n = n0 + wn * TN + j * 16 + nl + r;
          if (ml == 0 && n < p.N) { atomicAdd(st + n, s); atomicAdd(st + p.N + n, q); }
        }
    }
    __syncthreads();
    bf16* C = (bf16*)p.C + bz * p.sC;
    constexpr int CPR = BN / 8, TOT = BM * CPR;
    constexpr bool bnr = (EPI == EPI_BF16_BNR);
    const int ccol = tid % CPR;  // this thread's 8-column chunk (fixed: NT % CPR == 0)
    float r0[8], r1[8], r2[8], mu[8], is[8], sc[8], sh[8], mu2[8], is2[8];
    if constexpr (bnr) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int n = min(n0 + ccol * 8 + e, p.N - 1);
        r0[e] = r1[e] = r2[e] = 0.f;
        mu[e] = p.bn_mean[n]; is[e] = p.bn_invstd[n];
        sc[e] = p.bn_scale ? p.bn_scale[n] : 1.f; sh[e] = p.bn_shift ? p.bn_shift[n] : 0.f;
        mu2[e] = p.bn_y2 ? p.bn_mean2[n] : 0.f; is2[e] = p.bn_y2 ? p.bn_invstd2[n] : 0.f;
      }
    }
#pragma unroll
    for (int it = 0; it < TOT / NT; ++it) {
      const int idx = tid + it * NT;
      const int row = idx / CPR, cc = idx - row * CPR;
      const int m = m0 + row, n = n0 + cc * 8;
      if (m >= p.M || n >= p.N) continue;
      bf16x8 v = *(const bf16x8*)(Cs + row * LDC_S + cc * 8);
      bf16* dst = C + (long long)m * p.ldc + n;
      if (n + 7 < p.N && (p.ldc & 7) == 0) {
        const long long off = bz * p.sC + (long long)m * p.ldc + n;
        if constexpr (EPI == EPI_BF16_EXT) {
          // pre-activation chunk: [* act'(z)] -> [aux copy] -> act -> [dropout]; 16-B coalesced
          float f[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) f[e] = bf2f(v[e]);
          if (p.dact_src) {
            bf16x8 zv = *(const bf16x8*)((const bf16*)p.dact_src + off);
#pragma unroll
            for (int e = 0; e < 8; ++e) f[e] *= act_grad(bf2f(zv[e]), p.dact);
          }
          if (p.aux) *(bf16x8*)((bf16*)p.aux + off) = v;
#pragma unroll
          for (int e = 0; e < 8; ++e) f[e] = act_apply(f[e], p.act);
          if (p.drop_p > 0.f) {
            const unsigned long long lin = (unsigned long long)m * p.N + n;
#pragma unroll
            for (int e = 0; e < 8; ++e)
              f[e] = u01(hash_u32(p.drop_seed, lin + e)) < 1.f - p.drop_p ? f[e] * p.drop_scale : 0.f;
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = f2bf(f[e]);
        }
        if (p.resid) {
          bf16x8 rr = *(const bf16x8*)((const bf16*)p.resid + off);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = f2bf(bf2f(v[e]) + bf2f(rr[e]));
        }
        *(bf16x8*)dst = v;
        if constexpr (bnr) {
          bf16x8 yv = *(const bf16x8*)((const bf16*)p.bn_y + off);
          bf16x8 av, y2v;
          if (p.bn_a) av = *(const bf16x8*)((const bf16*)p.bn_a + off);
          if (p.bn_y2) y2v = *(const bf16x8*)((const bf16*)p.bn_y2 + off);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float y = bf2f(yv[e]);
            bool keep = p.bn_a ? (bf2f(av[e]) > 0.f) : (p.bn_relu ? (y * sc[e] + sh[e] > 0.f) : true);
            const float dz = keep ? bf2f(v[e]) : 0.f;
            r0[e] += dz;
            r1[e] += dz * (y - mu[e]) * is[e];
            if (p.bn_y2) r2[e] += dz * (bf2f(y2v[e]) - mu2[e]) * is2[e];
          }
        }
      } else {
        for (int e = 0; e < 8 && n + e < p.N; ++e) {
          const long long off = bz * p.sC + (long long)m * p.ldc + n + e;
          float x = bf2f(v[e]);
          if constexpr (EPI == EPI_BF16_EXT) {
            if (p.dact_src) x *= act_grad(bf2f(((const bf16*)p.dact_src)[off]), p.dact);
            if (p.aux) ((bf16*)p.aux)[off] = v[e];
            x = act_apply(x, p.act);
            if (p.drop_p > 0.f)
              x = u01(hash_u32(p.drop_seed, (unsigned long long)m * p.N + n + e)) < 1.f - p.drop_p ? x * p.drop_scale : 0.f;
            x = bf2f(f2bf(x));
          }
          if (p.resid) x += bf2f(((const bf16*)p.resid)[off]);
          dst[e] = f2bf(x);
        }
      }
    }
    if constexpr (bnr) {
      // lanes sharing a column chunk: tid % CPR equal -> xor over the bits above log2(CPR)
#pragma unroll
      for (int e = 0; e < 8; ++e)
#pragma unroll
        for (int o = CPR; o < 64; o <<= 1) {
          r0[e] += __shfl_xor(r0[e], o, 64);
          r1[e] += __shfl_xor(r1[e], o, 64);
          r2[e] += __shfl_xor(r2[e], o, 64);
        }
      __syncthreads();  // C tile no longer needed: reuse LDS for the cross-wave reduction
      float* red = (float*)smem;  // [NW waves][3][CPR*8]
      if (lane < CPR) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          red[(wid * 3 + 0) * (CPR * 8) + lane * 8 + e] = r0[e];
          red[(wid * 3 + 1) * (CPR * 8) + lane * 8 + e] = r1[e];
          red[(wid * 3 + 2) * (CPR * 8) + lane * 8 + e] = r2[e];
        }
      }
      __syncthreads();
      const int nsum = p.bn_y2 ? 3 : 2;
      float* st = p.bn_sums + (long long)(blockIdx.x % p.bn_shards) * 3 * p.N;
      for (int k = tid; k < nsum * CPR * 8; k += NT) {
        const int which = k / (CPR * 8), col = k - which * (CPR * 8);
        const int n = n0 + col;
        if (n >= p.N) continue;
        float v = 0.f;
#pragma unroll
        for (int w = 0; w < NW; ++w) v += red[(w * 3 + which) * (CPR * 8) + col];
        atomicAdd(st + which * p.N + n, v);
      }
    }
  }
}

}  // namespace tfk

using namespace tfk;

#define TFK_GEMM_CASE(BM_, BN_, AM_, BM2_, EPI_)                                                  \
  if (bm == BM_ && bn == BN_ && amode == AM_ && bmode == BM2_ && epi == EPI_) {                  \
    hipLaunchKernelGGL((gemm_kernel<BM_, BN_, AM_, BM2_, EPI_>), grid, dim3((threads_for<BM_, BN_>())), 0, stream, p); \
    return hipGetLastError() == hipSuccess ? 0 : -2;                                              \
  }
#define TFK_GEMM_TILES(AM_, BM2_, EPI_) \
  TFK_GEMM_CASE(128, 128, AM_, BM2_, EPI_) TFK_GEMM_CASE(128, 64, AM_, BM2_, EPI_) TFK_GEMM_CASE(64, 64, AM_, BM2_, EPI_)
// + the 256x256 (8-wave) tile for the dense (non-gather) operand modes
#define TFK_GEMM_TILES_BIG(AM_, BM2_, EPI_) TFK_GEMM_TILES(AM_, BM2_, EPI_) TFK_GEMM_CASE(256, 256, AM_, BM2_, EPI_)

// Host launcher. Grid: x = tiles (M x N), y = batch, z = split-K. Returns 0 on success.
extern "C" int tfk_gemm_launch(GemmParams p, int bm, int bn, int amode, int bmode, int epi, int batch, int splits,
                               hipStream_t stream) {
  const int tiles_m = (p.M + bm - 1) / bm, tiles_n = (p.N + bn - 1) / bn;
  const int nkt = (p.K + BK - 1) / BK;
  if (splits < 1) splits = 1;
  if (splits > nkt) splits = nkt > 0 ? nkt : 1;
  p.kt_per_split = (nkt + splits - 1) / splits;
  splits = nkt > 0 ? (nkt + p.kt_per_split - 1) / p.kt_per_split : 1;
  p.tiles_n = tiles_n;
  if (p.stats_shards < 1) p.stats_shards = 1;
  dim3 grid(tiles_m * tiles_n, batch, splits);
  if (epi == EPI_BF16 && p.bn_sums) epi = EPI_BF16_BNR;
  if (epi == EPI_BF16 && (p.aux || p.dact_src || p.drop_p > 0.f)) epi = EPI_BF16_EXT;
  TFK_GEMM_TILES_BIG(A_KIN, B_KIN, EPI_BF16)
  TFK_GEMM_TILES_BIG(A_KIN, B_KIN, EPI_F32)
  TFK_GEMM_TILES_BIG(A_KIN, B_KOUT, EPI_BF16)
  TFK_GEMM_TILES_BIG(A_KIN, B_KOUT, EPI_F32)
  TFK_GEMM_TILES_BIG(A_KOUT, B_KOUT, EPI_F32)
  TFK_GEMM_TILES_BIG(A_KOUT, B_KOUT, EPI_BF16)
  TFK_GEMM_TILES(A_CONV_FWD, B_KIN, EPI_BF16)
  TFK_GEMM_TILES(A_CONV_DGRAD, B_KIN, EPI_BF16)
  TFK_GEMM_TILES(A_CONV_DGRAD, B_KOUT, EPI_BF16)
  TFK_GEMM_TILES(A_KOUT, B_CONV_WGRAD, EPI_F32)
  // transformer epilogue extras: fwd (aux/dropout) and dgrad (activation backward)
  TFK_GEMM_TILES_BIG(A_KIN, B_KIN, EPI_BF16_EXT)
  TFK_GEMM_TILES_BIG(A_KIN, B_KOUT, EPI_BF16_EXT)
  // fused BN-backward reduction: only the dgrad producers of a BN input
  TFK_GEMM_TILES_BIG(A_KIN, B_KOUT, EPI_BF16_BNR)
  TFK_GEMM_TILES(A_CONV_DGRAD, B_KIN, EPI_BF16_BNR)
  TFK_GEMM_TILES(A_CONV_DGRAD, B_KOUT, EPI_BF16_BNR)
  return -1;  // unsupported combination
}

// Number of split-K slabs the launcher will actually use (for workspace sizing).
extern "C" int tfk_gemm_splits(int K, int splits) {
  const int nkt = (K + BK - 1) / BK;
  if (splits < 1) splits = 1;
  if (splits > nkt) splits = nkt > 0 ? nkt : 1;
  int per = (nkt + splits - 1) / splits;
  return nkt > 0 ? (nkt + per - 1) / per : 1;
}
