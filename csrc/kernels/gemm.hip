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
#include "gemm_epilogue.h"

namespace tfk {

enum AMode { A_KIN = 0, A_KOUT = 1, A_CONV_FWD = 2, A_CONV_DGRAD = 3 };
enum BMode { B_KIN = 0, B_KOUT = 1, B_CONV_WGRAD = 2 };


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

// Tile walk. One-shot grid (gridDim.x == tiles): the XCD remap. Persistent grid (gridDim.x <
// tiles, a multiple of 8 sized to the resident block count): block b serves a contiguous tile range
// of its XCD (b & 7 under round-robin dispatch), striding by that XCD's block count, so the blocks
// of one XCD walk neighbouring tiles together (shared A panels stay in that XCD's L2).
struct TileWalk {
  int cur, end, step;
  __device__ __forceinline__ explicit TileWalk(int ntiles) {
    const int G = gridDim.x, b = blockIdx.x;
    if (G >= ntiles) {
      cur = xcd_remap(b, G); end = cur + 1; step = 1;
    } else {
      const int x = b & 7, q = ntiles >> 3, r = ntiles & 7;
      const int start = x * q + (x < r ? x : r);
      cur = start + (b >> 3); end = start + q + (x < r ? 1 : 0); step = G >> 3;
    }
  }
};

template <int BM, int BN, int AM, int BMD, int EPI>
__global__ __launch_bounds__((threads_for<BM, BN>()), (threads_for<BM, BN>() == 512 ? 1 : 2)) void gemm_kernel(GemmParams p) {
  constexpr int NT = threads_for<BM, BN>();
  // Persistent walk over several tiles: the next tile's first K-tile is loaded into registers
  // before this tile's last MFMAs and stays in flight through the epilogue, so a short-K
  // (memory-bound) GEMM keeps HBM busy while it stores. The 8-wave 256x256 tile (long-K GEMMs,
  // one block per CU, no registers to spare) stays one-shot.
  // Dense A operands only: the conv gathers keep per-chunk geometry in registers and have none
  // left for an in-flight next tile (they spill); their GEMMs are long-K (3x3) or strided anyway.
  // (256x64 with the BN-backward epilogue: one-shot, its row maps + 8-chunk A prefetch spill)
  constexpr bool PERSIST = NT == 256 && (AM == A_KIN || AM == A_KOUT) && !(BM == 256 && EPI == EPI_BF16_BNR);
  constexpr int NW = NT / 64;                    // waves
  constexpr int WM = 2, WN = NW / WM;            // wave grid
  constexpr int TM = BM / WM, TN = BN / WN;      // wave tile
  constexpr int FM = TM / 16, FN = TN / 16;      // 16x16 fragments per wave
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  constexpr bool A_KOUT_ = (AM == A_KOUT);
  constexpr bool B_KOUT_ = (BMD == B_KOUT || BMD == B_CONV_WGRAD);
  constexpr int MAIN_BYTES = 2 * (A_BYTES + B_BYTES);
  constexpr int EPI_BYTES = (EPI == EPI_F32) ? 0 : epi_lds_bytes<BM, BN, WM>();
  __shared__ __attribute__((aligned(16))) char smem[MAIN_BYTES > EPI_BYTES ? MAIN_BYTES : EPI_BYTES];
  char* As = smem;
  char* Bs = smem + 2 * A_BYTES;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int bz = blockIdx.y;
  const bf16* Ab = (const bf16*)p.A + bz * p.sA;
  const bf16* Bb = (const bf16*)p.B + bz * p.sB;

  const int nkt = (p.K + BK - 1) / BK;
  const int kt0 = blockIdx.z * p.kt_per_split;
  const int kt1 = min(nkt, kt0 + p.kt_per_split);  // the launcher gives every split >= 1 K-tile

  TileWalk walk(((p.M + BM - 1) / BM) * p.tiles_n);
  if (walk.cur >= walk.end) return;  // block-uniform
  int m0 = (walk.cur / p.tiles_n) * BM, n0 = (walk.cur % p.tiles_n) * BN;

  Loader<BM, AM, true, NT> la;
  Loader<BN, BMD, false, NT> lb;
  la.S_ = p.S; lb.S_ = p.S;
  la.init(p, Ab, p.lda, m0, p.M, kt0);
  lb.init(p, Bb, p.ldb, n0, p.N, kt0);
  u32x4 ra[Loader<BM, AM, true, NT>::NCH], rb[Loader<BN, BMD, false, NT>::NCH];
  la.load(p, kt0, m0, ra);
  lb.load(p, kt0, n0, rb);

  for (;;) {
    la.store_lds(As, ra);
    lb.store_lds(Bs, rb);
    __syncthreads();

    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nxt = walk.cur + walk.step;
    const bool has_next = PERSIST && nxt < walk.end;
    const int nm0 = (nxt / p.tiles_n) * BM, nn0 = (nxt % p.tiles_n) * BN;

    for (int kt = kt0; kt < kt1; ++kt) {
      const int cur = (kt - kt0) & 1;
      const bool more = kt + 1 < kt1;
      if (more) {
        if constexpr (AM == A_CONV_FWD) la.advance(p.Cin);
        if constexpr (AM == A_CONV_DGRAD) la.advance(p.Cout);
        la.load(p, kt + 1, m0, ra);
        lb.load(p, kt + 1, n0, rb);
      } else if (has_next) {
        // issue-early: the next tile's first K-tile flies during the last MFMAs + epilogue
        la.init(p, Ab, p.lda, nm0, p.M, kt0);
        lb.init(p, Bb, p.ldb, nn0, p.N, kt0);
        la.load(p, kt0, nm0, ra);
        lb.load(p, kt0, nn0, rb);
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

    gemm_epilogue<BM, BN, NT, WM, EPI>(p, acc, smem, m0, n0, bz);
    if (!has_next) break;
    walk.cur = nxt; m0 = nm0; n0 = nn0;
    __syncthreads();  // every wave is done reading the epilogue's LDS before stage 0 is rewritten
  }
}

}  // namespace tfk

using namespace tfk;

// Persistent grids on (default) unless TFK_GEMM_PERSIST=0 or tfk_gemm_set_persist(0).
static int g_persist = -1;
static bool persist_on() {
  if (g_persist < 0) {
    const char* e = getenv("TFK_GEMM_PERSIST");
    g_persist = (e && e[0] == '0') ? 0 : 1;
  }
  return g_persist == 1;
}
extern "C" void tfk_gemm_set_persist(int on) { g_persist = on ? 1 : 0; }

// Launch one instantiation. 4-wave tiles with more tiles than resident blocks get a persistent
// grid of exactly the resident count (occupancy query, cached per instantiation; a multiple of 8
// so TileWalk's XCD split holds).
template <int BM_, int BN_, int AM_, int BM2_, int EPI_>
static int launch_gemm(const GemmParams& p, int tiles, int batch, int splits, hipStream_t stream) {
  constexpr int NT = threads_for<BM_, BN_>();
  int gx = tiles;
  constexpr bool can_persist = NT == 256 && (AM_ == A_KIN || AM_ == A_KOUT) && !(BM_ == 256 && EPI_ == EPI_BF16_BNR);
  if (can_persist && persist_on()) {
    static int resident = 0;
    if (resident == 0) {
      int dev = 0, cus = 0, per_cu = 0;
      if (hipGetDevice(&dev) == hipSuccess &&
          hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
          hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, gemm_kernel<BM_, BN_, AM_, BM2_, EPI_>, NT, 0) ==
              hipSuccess &&
          cus > 0 && per_cu > 0)
        resident = (cus * per_cu) & ~7;
      else
        resident = -1;
    }
    if (resident >= 8 && tiles > resident) gx = resident;
  }
  hipLaunchKernelGGL((gemm_kernel<BM_, BN_, AM_, BM2_, EPI_>), dim3(gx, batch, splits), dim3(NT), 0, stream, p);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

#define TFK_GEMM_CASE(BM_, BN_, AM_, BM2_, EPI_)                                 \
  if (bm == BM_ && bn == BN_ && amode == AM_ && bmode == BM2_ && epi == EPI_) { \
    return launch_gemm<BM_, BN_, AM_, BM2_, EPI_>(p, tiles_m * tiles_n, batch, splits, stream); \
  }
// gather A modes (conv fwd/dgrad): 3 tiles (a 256-row gather tile needs more registers than exist)
#define TFK_GEMM_TILES3(AM_, BM2_, EPI_) \
  TFK_GEMM_CASE(128, 128, AM_, BM2_, EPI_) TFK_GEMM_CASE(128, 64, AM_, BM2_, EPI_) TFK_GEMM_CASE(64, 64, AM_, BM2_, EPI_)
// + the 256x64 tile (narrow-N GEMMs: twice the MFMA work per K-tile barrier of 128x64)
#define TFK_GEMM_TILES(AM_, BM2_, EPI_) TFK_GEMM_TILES3(AM_, BM2_, EPI_) TFK_GEMM_CASE(256, 64, AM_, BM2_, EPI_)
#define TFK_GEMM_TILES_BIG(AM_, BM2_, EPI_) TFK_GEMM_TILES(AM_, BM2_, EPI_) TFK_GEMM_CASE(256, 256, AM_, BM2_, EPI_)

extern "C" int tfk_g4_ok(const GemmParams& p, int amode, int bmode);
extern "C" int tfk_g4_launch(const GemmParams& p, int bm, int bn, int amode, int bmode, int epi, int batch, int splits,
                             hipStream_t stream);
// Engine for the tiles the LDS-DMA kernel serves: 1 = g4 (gemm_g4.hip: 64x64 wave tiles,
// 128x128 / 256x256 blocks, dense + conv-fwd gather), 0 = this file's register-staged engine
// (TFK_GEMM_ENGINE=reg, for A/B).
static int g_pp = -1;
static int engine() {
  if (g_pp < 0) {
    const char* e = getenv("TFK_GEMM_ENGINE");
    g_pp = (e && e[0] == 'r') ? 0 : 1;
  }
  return g_pp;
}
extern "C" void tfk_gemm_set_engine(int e) { g_pp = e; }

// Host launcher. Grid: x = tiles (M x N), y = batch, z = split-K. Returns 0 on success.
// Register-staged engine: every instantiated (tile, operand modes, epilogue). -1 if absent.
static int launch_reg(GemmParams p, int bm, int bn, int amode, int bmode, int epi, int batch, int splits,
                      hipStream_t stream) {
  const int tiles_m = (p.M + bm - 1) / bm, tiles_n = (p.N + bn - 1) / bn;
  p.tiles_n = tiles_n;
  TFK_GEMM_TILES_BIG(A_KIN, B_KIN, EPI_BF16)
  TFK_GEMM_TILES_BIG(A_KIN, B_KIN, EPI_F32)
  TFK_GEMM_TILES_BIG(A_KIN, B_KOUT, EPI_BF16)
  TFK_GEMM_TILES_BIG(A_KIN, B_KOUT, EPI_F32)
  TFK_GEMM_TILES_BIG(A_KOUT, B_KOUT, EPI_F32)
  TFK_GEMM_TILES3(A_KOUT, B_KOUT, EPI_BF16) TFK_GEMM_CASE(256, 256, A_KOUT, B_KOUT, EPI_BF16)
  TFK_GEMM_TILES3(A_CONV_FWD, B_KIN, EPI_BF16)
  // activated bf16 outputs without the EXT extras (inference linears, conv + relu without a BN)
  TFK_GEMM_TILES3(A_KIN, B_KIN, EPI_BF16_ACT)
  TFK_GEMM_TILES3(A_CONV_FWD, B_KIN, EPI_BF16_ACT)
  TFK_GEMM_TILES3(A_CONV_DGRAD, B_KIN, EPI_BF16)
  TFK_GEMM_TILES3(A_CONV_DGRAD, B_KOUT, EPI_BF16)
  TFK_GEMM_TILES(A_KOUT, B_CONV_WGRAD, EPI_F32)
  // Cout=64 conv weight gradients (stem 7x7, stage-1 3x3): a 64x256 tile gives each wave a 32x128
  // sub-tile (2x8 MFMA fragments per LDS fragment load instead of 64x64's 2x2)
  TFK_GEMM_CASE(64, 256, A_KOUT, B_CONV_WGRAD, EPI_F32)
  // transformer epilogue extras: fwd (aux/dropout) and dgrad (activation backward). Register-engine
  // fallback only (g4 serves every aligned shape); the 256x64 tiles and the 128x128 K-outer-B tile
  // spill with this epilogue (8-32 B/lane of scratch under hipcc 7.2), so they are not built -- the
  // launcher falls back to 128x64 / 64x64 for them.
  TFK_GEMM_TILES3(A_KIN, B_KIN, EPI_BF16_EXT) TFK_GEMM_CASE(256, 256, A_KIN, B_KIN, EPI_BF16_EXT)
  TFK_GEMM_CASE(128, 64, A_KIN, B_KOUT, EPI_BF16_EXT) TFK_GEMM_CASE(64, 64, A_KIN, B_KOUT, EPI_BF16_EXT)
  TFK_GEMM_CASE(256, 256, A_KIN, B_KOUT, EPI_BF16_EXT)
  // fused BN-backward reduction: only the dgrad producers of a BN input
  TFK_GEMM_TILES_BIG(A_KIN, B_KOUT, EPI_BF16_BNR)
  TFK_GEMM_TILES3(A_CONV_DGRAD, B_KIN, EPI_BF16_BNR)
  TFK_GEMM_TILES3(A_CONV_DGRAD, B_KOUT, EPI_BF16_BNR)
  return -1;  // unsupported combination
}

// Host launcher. Grid: x = tiles (M x N), y = batch, z = split-K. Returns 0 on success.
// The LDS-DMA engine (g4) takes the tiles/modes it serves; the rest, and any tile it declines
// (ineligible shape/alignment), runs on the register-staged engine.
extern "C" int tfk_gemm_launch(GemmParams p, int bm, int bn, int amode, int bmode, int epi, int batch, int splits,
                               hipStream_t stream) {
  const int nkt = (p.K + BK - 1) / BK;
  if (splits < 1) splits = 1;
  if (splits > nkt) splits = nkt > 0 ? nkt : 1;
  p.kt_per_split = (nkt + splits - 1) / splits;
  splits = nkt > 0 ? (nkt + p.kt_per_split - 1) / p.kt_per_split : 1;
  p.tiles_n = (p.N + bn - 1) / bn;
  if (p.stats_shards < 1) p.stats_shards = 1;
  if (epi == EPI_BF16 && p.bn_sums) epi = EPI_BF16_BNR;
  if (epi == EPI_BF16 && (p.aux || p.dact_src || p.drop_p > 0.f)) epi = EPI_BF16_EXT;
  if (p.act != 0 && epi == EPI_BF16_BNR) return -3;  // no activated output feeds a BN-backward reduction
  if (epi == EPI_BF16 && p.act != 0) epi = EPI_BF16_ACT;  // EPI_BF16's epilogue is activation-free
  // row maps (strided-conv dgrad phases, lattice residual) live in the BN-reduce epilogue, which
  // both engines share
  if ((p.om_hp == 0 && p.rs_sh == 0) || epi == EPI_BF16_BNR) {
    if (engine() == 1 && tfk_g4_ok(p, amode, bmode)) {
      const int r = tfk_g4_launch(p, bm, bn, amode, bmode, epi, batch, splits, stream);
      if (r != -1) return r;
    }
  }
  // requested tile, else the 128x128 / 128x64 / 64x64 tiles every combination instantiates at
  // least one of
  int r = launch_reg(p, bm, bn, amode, bmode, epi, batch, splits, stream);
  const int fb[3][2] = {{128, 128}, {128, 64}, {64, 64}};
  for (int i = 0; i < 3 && r == -1; ++i)
    if (!(bm == fb[i][0] && bn == fb[i][1])) r = launch_reg(p, fb[i][0], fb[i][1], amode, bmode, epi, batch, splits, stream);
  return r;
}

// Number of split-K slabs the launcher will actually use (for workspace sizing).
extern "C" int tfk_gemm_splits(int K, int splits) {
  const int nkt = (K + BK - 1) / BK;
  if (splits < 1) splits = 1;
  if (splits > nkt) splits = nkt > 0 ? nkt : 1;
  int per = (nkt + splits - 1) / splits;
  return nkt > 0 ? (nkt + per - 1) / per : 1;
}
