// Fused multi-head attention (flash style) for gfx950: forward, dQ pass, dK/dV pass.
//
// Head dim D = 64. Q/K/V/O/dO are bf16 [B, S, H, 64] views with arbitrary token (row) and batch
// strides, so Q, K and V can be read straight out of a fused QKV projection ([B*S, 3*H*64]) and O
// is written in the [B*S, H*64] layout the output projection consumes: no head transposes.
// lse/delta are f32 [B, H, Sq]. Options: causal mask, per-batch key length (padding mask),
// attention-probability dropout (hash RNG of (seed, b, h, q, key) regenerated in backward).
//
// MFMA mapping (v_mfma_f32_16x16x32_bf16, wave64). mfma(X, Y) gives lane l, slot r:
//   sum_k X[4*(l>>4) + r][k] * Y[l & 15][k]
// where an operand fragment puts row (l & 15), k-slots 8*(l>>4)..+7 in lane l. Rows of Q (or K in
// the dK/dV pass) stay lane-fixed ((l&15) = query), so softmax statistics are per-lane scalars and
// row reductions are 4 register values + 2 shuffles. Within each 32-key chunk the 16-row blocks
// of the "X" operand are read with the row permutation  i -> 8*(i>>2) + 4*half + (i&3)  so that
// the P / dS accumulators of two blocks, packed to bf16, are directly the k-slots 8g..8g+7 of the
// next MFMA (P*V, dS*K, ...) whose other operand is a transposed LDS read (ds_read_b64_tr_b16).
// LDS tiles are [64 rows][64] bf16 with XOR-swizzled 16-B chunks (aswz: conflict-free row and tr reads).
//
// Backward = two kernels (no atomics, deterministic): dQ pass (grid over query tiles, recompute
// P and dP, dQ = dS K) and dK/dV pass (grid over key tiles, dV = P^T dO, dK = dS^T Q).
#include "common.h"
#include <type_traits>

namespace {
constexpr int D = 64;
constexpr int TILE = 64;
constexpr int LS = 64;  // LDS row stride (elements): 128-B rows, 16-B chunks XOR-swizzled (aswz)
// chunk c of tile row r sits at chunk position c ^ aswz(r). With gfx950's ds_read_b128 lane groups
// ({0-3,12-15,20-27}, ...) and the permuted rows of frag_row, and the 32-lane groups of
// ds_read_b64_tr_b16 in frag_tr, this is conflict-free for both reads (a 144-B padded row -- the r3
// layout -- costs 2x: SQ_LDS_BANK_CONFLICT 2.1e6 / 3.1e6 / 4.2e6 cycles per fwd / dQ / dKV call).
// (independent of row bit 2, so rows r and r + 4 share it: the +4-row fragment reads are immediate
// offsets of the same per-lane base)
__device__ __forceinline__ int aswz(int r) { return (((r >> 2) & 6) ^ ((r & 3) << 1)) & 7; }
constexpr int NT = 256;
constexpr float LOG2E = 1.4426950408889634f;

struct AttnParams {
  const bf16 *q, *k, *v, *o, *dout;
  bf16 *out, *dq, *dk, *dv;
  float *lse, *delta;
  long long q_bs, k_bs, v_bs, o_bs, dq_bs, dk_bs, dv_bs;  // batch strides (elements)
  int q_rs, k_rs, v_rs, o_rs, dq_rs, dk_rs, dv_rs;        // token strides (elements)
  int B, H, Sq, Sk;
  const int* kv_len;  // [B] valid keys per batch (padding mask) or null
  float scale;
  int causal;
  float p_drop;
  unsigned long long seed;         // per-site salt
  const unsigned long long* seed_key;  // per-step device key (common.h eff_seed) or null
};

__device__ __forceinline__ f32x4 mfma(bf16x8 x, bf16x8 y, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, y, c, 0, 0, 0);
}

// permuted row of 16-row block b inside a 64-row tile for lane-row i (see header)
__device__ __forceinline__ int prow(int b, int i) { return 32 * (b >> 1) + 8 * (i >> 2) + 4 * (b & 1) + (i & 3); }
// tile-relative row held by accumulator slot r of lane group g for block b
__device__ __forceinline__ int arow(int b, int g, int r) { return 32 * (b >> 1) + 8 * g + 4 * (b & 1) + r; }

// ---- global tile <-> registers <-> LDS (64 rows x 64 bf16; 2 x 16 B per thread)
struct TileRegs {
  u32x4 v[2];
  bool ok[2];
};
// Loads are unconditional (rows past nvalid re-read the last valid row, or row 0) and the padding zeros
// are applied when the registers are stored: no exec-masked branch around the loads, so the
// compiler's wait for them stays at the store, a whole tile later.
template <int NTH>  // NTH <= 512: a 64 x 64 tile is 512 16-B chunks
__device__ __forceinline__ void tile_load(TileRegs& t, const bf16* base, int rs, int row0, int nvalid) {
#pragma unroll
  for (int it = 0; it < 512 / NTH; ++it) {
    const int c = threadIdx.x + it * NTH, row = c >> 3, col = (c & 7) * 8;
    t.ok[it] = row0 + row < nvalid;
    // 32-bit byte offset from the block-uniform base: the SGPR-base + VGPR-offset load form (a
    // head's rows span < 4 GiB), no 64-bit per-lane address pairs held across the loop
    const unsigned off = (unsigned)(max(min(row0 + row, nvalid - 1), 0) * rs + col) * 2u;
    t.v[it] = *(const u32x4*)((const char*)base + off);
  }
}
template <int NTH>
__device__ __forceinline__ void tile_store(const TileRegs& t, bf16* lds) {
#pragma unroll
  for (int it = 0; it < 512 / NTH; ++it) {
    const int c = threadIdx.x + it * NTH, row = c >> 3, col = (c & 7) * 8;
    const u32x4 z = u32x4{0u, 0u, 0u, 0u};
    *(u32x4*)(lds + row * LS + (((col >> 3) ^ aswz(row)) << 3)) = t.ok[it] ? t.v[it] : z;
  }
}
// Per-lane LDS byte offsets of the fragment reads, computed once per kernel (the swizzle is a
// lane-dependent XOR, so the compile-time parts -- k-half, block parity, column block -- select one
// of a few precomputed offsets and the remaining row shifts are immediate offsets):
//  frag_row (row prow(bb, l&15), k-slots kk*32 + 8g..+7): row[kk] + 4*(bb&1) + 32*(bb>>1) rows,
//    since aswz(r + 4) == aswz(r + 32) == aswz(r);
//  frag_tr (column cbase + (l&15), k-slots = tile rows kbase + 8g..+7, two 4-row reads): tr[cbase/16]
//    + kbase rows (+ 4 rows for the second read; kbase in {0, 32}).
struct FragOffs {
  int row[2];
  int tr[4];
  __device__ __forceinline__ void init() {
    const int l = threadIdx.x & 63, g = l >> 4, li = l & 15;
    const int R0 = 8 * (li >> 2) + (li & 3);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) row[kk] = R0 * 128 + (((kk * 4 + g) ^ aswz(R0)) << 4);
    const int qq = li >> 2, pc = li & 3, r = 8 * g + qq;
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      const int col = cb * 16 + 4 * pc;
      tr[cb] = r * 128 + (((col >> 3) ^ aswz(r)) << 4) + (col & 7) * 2;
    }
  }
};
// row fragment of block bb: lane -> tile row prow(bb, l&15), k-slots kk*32 + 8g .. +7
__device__ __forceinline__ bf16x8 frag_row(const bf16* lds, const FragOffs& o, int bb, int kk) {
  return *(const bf16x8*)((const char*)lds + o.row[kk] + ((bb & 1) * 4 + (bb >> 1) * 32) * 128);
}
// transposed fragment: lane -> column cbase + (l&15), k-slots = tile rows kbase + 8g .. +7
__device__ __forceinline__ bf16x8 frag_tr(const bf16* lds, const FragOffs& o, int kbase, int cbase) {
  const char* b = (const char*)lds + kbase * 128;
  bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((LDS_AS bf16x4*)(b + o.tr[cbase >> 4]));
  bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((LDS_AS bf16x4*)(b + o.tr[cbase >> 4] + 4 * 128));
  bf16x8 r;
  r.lo = lo;
  r.hi = hi;
  return r;
}
// register row fragment straight from global (rows of this wave): row `row` (global), k-slots kk;
// unconditional load of a clamped row, zeroed past nvalid
__device__ __forceinline__ bf16x8 frag_global(const bf16* base, int rs, int row, int nvalid, int kk) {
  const int g = (threadIdx.x & 63) >> 4;
  const bf16x8 v = *(const bf16x8*)(base + (long long)max(min(row, nvalid - 1), 0) * rs + kk * 32 + 8 * g);
  const u32x4 z = u32x4{0u, 0u, 0u, 0u};
  const u32x4 r = row < nvalid ? __builtin_bit_cast(u32x4, v) : z;
  return __builtin_bit_cast(bf16x8, r);
}
__device__ __forceinline__ bf16x8 pack2(const f32x4& a, const f32x4& b) {
  bf16x8 r;
#pragma unroll
  for (int e = 0; e < 4; ++e) { r[e] = f2bf(a[e]); r[4 + e] = f2bf(b[e]); }
  return r;
}
// keep iff the element's 24-bit uniform >= p_drop; element index q*Sk + key of head (b, h), the
// seed folded with the head index (ops/transformer.py dropout_keep_mask is the bit-exact reference)
__device__ __forceinline__ uint32_t head_seed(const AttnParams& p, int bh) {
  const unsigned long long s = eff_seed(p.seed, p.seed_key);
  return hash32((uint32_t)s ^ (uint32_t)(s >> 32) ^ ((uint32_t)bh * 0x9E3779B9u));
}
// Attention-probability dropout: ONE hash32 per (group of 4 queries, key) gives 4 mask bytes, byte
// j for query 4*qg + j; keep iff byte >= thr = round(p * 256) (keep scale 256 / (256 - thr)). In
// the forward / dQ kernels a lane owns one query and 4 consecutive keys, so a lane quad (the 4
// queries of a group) hashes its 4 keys once each and trades bytes over DPP quad broadcasts; in the
// dK/dV kernel a lane owns one key and 4 consecutive queries: one hash, 4 bytes. The per-element
// hash (plus its two quarter-rate multiplies) was the largest VALU cost of all three kernels.
// ops/transformer.py dropout_keep_mask is the bit-exact CPU copy.
__device__ __forceinline__ int drop_thr(float p) {
  const int t = (int)(p * 256.f + 0.5f);
  return t > 255 ? 255 : t;
}
template <int R>
__device__ __forceinline__ uint32_t qb(uint32_t h) {  // quad-broadcast lane R's h (DPP quad_perm [R,R,R,R])
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)h, R * 0x55, 0xf, 0xf, false);
}
// keep bits (bit r) of this lane's query (j = qrow & 3) with keys kb + r, r = 0..3 (kb % 4 == 0)
__device__ __forceinline__ unsigned keep4_rows(uint32_t hs, int qgbase, int kb, int j, int thr) {
  const uint32_t h = hash32(hs ^ (uint32_t)(qgbase + kb + j));
  const uint32_t h0 = qb<0>(h), h1 = qb<1>(h), h2 = qb<2>(h), h3 = qb<3>(h);
  const int sh = 8 * j;
  return (((h0 >> sh) & 0xffu) >= (uint32_t)thr ? 1u : 0u) | (((h1 >> sh) & 0xffu) >= (uint32_t)thr ? 2u : 0u) |
         (((h2 >> sh) & 0xffu) >= (uint32_t)thr ? 4u : 0u) | (((h3 >> sh) & 0xffu) >= (uint32_t)thr ? 8u : 0u);
}
// keep bits (bit r) of this lane's key with queries 4*qg + r
__device__ __forceinline__ unsigned keep4_cols(uint32_t hs, int qg, int Sk, int key, int thr) {
  const uint32_t h = hash32(hs ^ (uint32_t)(qg * Sk + key));
  return ((h & 0xffu) >= (uint32_t)thr ? 1u : 0u) | (((h >> 8) & 0xffu) >= (uint32_t)thr ? 2u : 0u) |
         (((h >> 16) & 0xffu) >= (uint32_t)thr ? 4u : 0u) | ((h >> 24) >= (uint32_t)thr ? 8u : 0u);
}
__device__ __forceinline__ void store_rowvec4(bf16* dst, const f32x4& v, float s) {
  bf16x4 o;
#pragma unroll
  for (int e = 0; e < 4; ++e) o[e] = f2bf(v[e] * s);
  *(bf16x4*)dst = o;
}

// v_exp_f32 without the libm denormal fix-up (exp2f adds a compare, two selects, an add and an
// ldexp): softmax terms below 2^-126 of the row maximum flush to 0
__device__ __forceinline__ float ex2(float x) { return __builtin_amdgcn_exp2f(x); }
// Butterfly reductions over the 4 lane rows (lanes l, l^16, l^32, l^48: the 4 k-groups of one
// query) with gfx950's v_permlane16/32_swap -- plain VALU, where __shfl_xor is an LDS bpermute plus
// an lgkmcnt(0) wait (4 per tile in the forward). swap(x, x) leaves (x[l], x[partner]) in the pair.
__device__ __forceinline__ float rows_max(float v) {
  auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
__device__ __forceinline__ float rows_sum(float v) {
  auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}
// LDS-only block barrier. __syncthreads() is a workgroup release/acquire fence around s_barrier and
// drains EVERY outstanding global load (vmcnt(0)) -- including the next tile's register prefetch,
// which must stay in flight across the barrier. The tiles only communicate through LDS, so waiting
// for this wave's LDS ops (lgkmcnt(0)) is enough.
__device__ __forceinline__ void lds_bar() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Occupancy: the 8-wave kernels are held to <= 128 VGPRs (waves_per_eu 4) so two 512-thread blocks
// share a CU (2 x 37 KiB of LDS); the backward kernels work on 32-row halves of each tile to fit.
// Every kernel stages its streamed 64-row tiles global -> registers -> LDS through a DOUBLE-buffered
// LDS ring with one barrier per tile: tile t+1 (loaded into registers during tile t-1) is stored
// into the idle buffer after tile t's math, and tile t+2's global loads are issued right behind it,
// so a whole tile of MFMA work covers each load.
//
// The kernels are VALU-issue bound (one v_exp and ~5-10 other VALU ops per score element against
// 1/16 of a 16x16x32 MFMA), so the element math is specialised: DROP (template: p_drop > 0) and
// FULL (per tile, wave-uniform: no mask needed) pick one of four straight-line bodies, instead of
// one body that evaluates the masks and both dropout arms for every element. The dropout keep
// scale is applied once per output row / accumulator instead of per element (O and dV are linear
// in the kept P; dS = P (dP_kept * scale - delta) is one FMA).
template <bool B>
using bconst = std::integral_constant<bool, B>;

// =============================================================================== forward
template <int NW, bool DROP>
__global__ __launch_bounds__(NW * 64, NW == 8 ? 4 : 2) void attn_fwd_kernel(AttnParams p) {
  constexpr int NTH = NW * 64, RB = 16 * NW;  // threads; query rows per block
  __shared__ __attribute__((aligned(16))) bf16 Ks[2][TILE * LS];
  __shared__ __attribute__((aligned(16))) bf16 Vs[2][TILE * LS];
  const int l = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), g = l >> 4, li = l & 15;
  FragOffs fo;
  fo.init();
  const int b = blockIdx.z, h = blockIdx.y, q0 = blockIdx.x * RB;
  const int bh = b * p.H + h;
  const uint32_t hs = head_seed(p, bh);
  const bf16* Qb = p.q + b * p.q_bs + h * D;
  const bf16* Kb = p.k + b * p.k_bs + h * D;
  const bf16* Vb = p.v + b * p.v_bs + h * D;
  const int kvl = p.kv_len ? min(p.kv_len[b], p.Sk) : p.Sk;
  const int qrow = q0 + 16 * w + li;  // this lane's query
  int kend = kvl;
  if (p.causal) kend = min(kend, q0 + RB);
  const int ntiles = (kend + TILE - 1) / TILE;
  TileRegs kr, vr;
  // prologue (unconditional: the tile-0 store's wait then covers every prologue load on all paths)
  tile_load<NTH>(kr, Kb, p.k_rs, 0, kvl);
  tile_load<NTH>(vr, Vb, p.v_rs, 0, kvl);
  const bf16x8 qf0 = frag_global(Qb, p.q_rs, qrow, p.Sq, 0), qf1 = frag_global(Qb, p.q_rs, qrow, p.Sq, 1);
  const float sl2 = p.scale * LOG2E;
  const int thr = drop_thr(p.p_drop);
  const float keep_scale = DROP ? 256.f / (float)(256 - thr) : 1.f;
  const int qgbase = (qrow >> 2) * p.Sk;
  float m = -INFINITY, lsum = 0.f;  // running max (log2 units) and row sum of the UNdropped P
  f32x4 oacc[4];
#pragma unroll
  for (int db = 0; db < 4; ++db) oacc[db] = f32x4{0.f, 0.f, 0.f, 0.f};
  tile_store<NTH>(kr, Ks[0]);
  tile_store<NTH>(vr, Vs[0]);
  tile_load<NTH>(kr, Kb, p.k_rs, TILE, kvl);
  tile_load<NTH>(vr, Vb, p.v_rs, TILE, kvl);
  lds_bar();
  for (int t = 0; t < ntiles; ++t) {
    const int k0 = t * TILE;
    const bf16* K_ = Ks[t & 1];
    const bf16* V_ = Vs[t & 1];
    // S^T blocks: lane (g, r) of block bb = score(key k0 + arow(bb,g,r), query qrow)
    f32x4 s[4];
#pragma unroll
    for (int bb = 0; bb < 4; ++bb) {
      f32x4 a = f32x4{0.f, 0.f, 0.f, 0.f};
      a = mfma(frag_row(K_, fo, bb, 0), qf0, a);
      a = mfma(frag_row(K_, fo, bb, 1), qf1, a);
      s[bb] = a;
    }
    // wave-uniform: every (query, key) of this wave's tile valid -> no per-element mask
    const bool full = k0 + TILE <= kvl && (!p.causal || k0 + TILE - 1 <= q0 + 16 * w);
    auto body = [&](auto FULL) {
      constexpr bool F = decltype(FULL)::value;
      // max over the RAW scores (scale > 0), masked ones -inf; exp2(s * sl2 - m) is one FMA + v_exp
      float mx = -INFINITY;
#pragma unroll
      for (int bb = 0; bb < 4; ++bb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (!F) {
            const int key = k0 + arow(bb, g, r);
            if (key >= kvl || (p.causal && key > qrow)) s[bb][r] = -INFINITY;
          }
          mx = fmaxf(mx, s[bb][r]);
        }
      mx = rows_max(mx);
      const float mnew = fmaxf(m, mx * sl2);
      const float muse = mnew == -INFINITY ? 0.f : mnew;
      const float alpha = ex2(m - muse);
      float rs = 0.f;
#pragma unroll
      for (int bb = 0; bb < 4; ++bb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float e = ex2(fmaf(s[bb][r], sl2, -muse));
          rs += e;
          s[bb][r] = e;
        }
      rs = rows_sum(rs);
      lsum = lsum * alpha + rs;
      m = mnew;
#pragma unroll
      for (int db = 0; db < 4; ++db) oacc[db] *= alpha;
      if (DROP) {
#pragma unroll
        for (int bb = 0; bb < 4; ++bb) {
          const unsigned kp = keep4_rows(hs, qgbase, k0 + arow(bb, g, 0), li & 3, thr);
#pragma unroll
          for (int r = 0; r < 4; ++r) s[bb][r] = (kp & (1u << r)) ? s[bb][r] : 0.f;
        }
      }
    };
    if (full) body(bconst<true>{});
    else body(bconst<false>{});
    const bf16x8 pf0 = pack2(s[0], s[1]), pf1 = pack2(s[2], s[3]);
#pragma unroll
    for (int db = 0; db < 4; ++db) {
      oacc[db] = mfma(frag_tr(V_, fo, 0, db * 16), pf0, oacc[db]);
      oacc[db] = mfma(frag_tr(V_, fo, 32, db * 16), pf1, oacc[db]);
    }
    // unconditional: past the end these stage clamped rows into the idle buffer, never read
    tile_store<NTH>(kr, Ks[(t + 1) & 1]);
    tile_store<NTH>(vr, Vs[(t + 1) & 1]);
    tile_load<NTH>(kr, Kb, p.k_rs, k0 + 2 * TILE, kvl);
    tile_load<NTH>(vr, Vb, p.v_rs, k0 + 2 * TILE, kvl);
    lds_bar();
  }
  if (qrow < p.Sq) {
    const float inv = lsum > 0.f ? keep_scale / lsum : 0.f;
    bf16* O = p.out + b * p.o_bs + (long long)qrow * p.o_rs + h * D;
#pragma unroll
    for (int db = 0; db < 4; ++db) store_rowvec4(O + db * 16 + 4 * g, oacc[db], inv);
    if (g == 0 && p.lse)
      p.lse[(long long)bh * p.Sq + qrow] = lsum > 0.f ? (m + log2f(lsum)) / LOG2E : INFINITY;
  }
}

// =============================================================================== dQ pass
template <int NW, bool DROP>
__global__ __launch_bounds__(NW * 64, NW == 8 ? 4 : 2) void attn_bwd_dq_kernel(AttnParams p) {
  constexpr int NTH = NW * 64, RB = 16 * NW;  // threads; query rows per block
  __shared__ __attribute__((aligned(16))) bf16 Ks[2][TILE * LS];
  __shared__ __attribute__((aligned(16))) bf16 Vs[2][TILE * LS];
  const int l = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), g = l >> 4, li = l & 15;
  FragOffs fo;
  fo.init();
  const int b = blockIdx.z, h = blockIdx.y, q0 = blockIdx.x * RB;
  const int bh = b * p.H + h;
  const uint32_t hs = head_seed(p, bh);
  const bf16* Qb = p.q + b * p.q_bs + h * D;
  const bf16* Kb = p.k + b * p.k_bs + h * D;
  const bf16* Vb = p.v + b * p.v_bs + h * D;
  const bf16* dOb = p.dout + b * p.o_bs + h * D;
  const int kvl = p.kv_len ? min(p.kv_len[b], p.Sk) : p.Sk;
  const int qrow = q0 + 16 * w + li;
  int kend = kvl;
  if (p.causal) kend = min(kend, q0 + RB);
  const int ntiles = (kend + TILE - 1) / TILE;
  TileRegs kr, vr;
  tile_load<NTH>(kr, Kb, p.k_rs, 0, kvl);
  tile_load<NTH>(vr, Vb, p.v_rs, 0, kvl);
  const bf16x8 qf0 = frag_global(Qb, p.q_rs, qrow, p.Sq, 0), qf1 = frag_global(Qb, p.q_rs, qrow, p.Sq, 1);
  const bf16x8 df0 = frag_global(dOb, p.o_rs, qrow, p.Sq, 0), df1 = frag_global(dOb, p.o_rs, qrow, p.Sq, 1);
  const float sl2 = p.scale * LOG2E;
  const int thr = drop_thr(p.p_drop);
  const float keep_scale = DROP ? 256.f / (float)(256 - thr) : 1.f;
  const int qgbase = (qrow >> 2) * p.Sk;
  const float lse2 = qrow < p.Sq ? p.lse[(long long)bh * p.Sq + min(qrow, p.Sq - 1)] * LOG2E : INFINITY;
  // delta = rowsum(dO * O) of this lane's query, from the dO fragments already in registers + the
  // same fragments of O (4 lane groups x 16 of the 64 dims); written for the dK/dV pass, which
  // runs after this kernel -- no separate delta kernel (a strided 128-B-per-lane pass)
  float dlt;
  {
    const bf16* Ob = p.o + b * p.o_bs + h * D;
    const bf16x8 of0 = frag_global(Ob, p.o_rs, qrow, p.Sq, 0), of1 = frag_global(Ob, p.o_rs, qrow, p.Sq, 1);
    float d = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) d += bf2f(df0[e]) * bf2f(of0[e]) + bf2f(df1[e]) * bf2f(of1[e]);
    d = rows_sum(d);
    dlt = d;
    if (g == 0 && qrow < p.Sq) p.delta[(long long)bh * p.Sq + qrow] = d;
  }
  f32x4 acc[4];
#pragma unroll
  for (int db = 0; db < 4; ++db) acc[db] = f32x4{0.f, 0.f, 0.f, 0.f};
  tile_store<NTH>(kr, Ks[0]);
  tile_store<NTH>(vr, Vs[0]);
  tile_load<NTH>(kr, Kb, p.k_rs, TILE, kvl);
  tile_load<NTH>(vr, Vb, p.v_rs, TILE, kvl);
  lds_bar();
  for (int t = 0; t < ntiles; ++t) {
    const int k0 = t * TILE;
    const bf16* K_ = Ks[t & 1];
    const bf16* V_ = Vs[t & 1];
    const bool full = k0 + TILE <= kvl && (!p.causal || k0 + TILE - 1 <= q0 + 16 * w);
    // two 32-key halves: S/dP of blocks 2hh, 2hh+1 -> dS -> its dQ MFMAs (k-slots 32hh..32hh+31)
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      f32x4 s[2], dp[2], ds[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        f32x4 a = f32x4{0.f, 0.f, 0.f, 0.f}, c = f32x4{0.f, 0.f, 0.f, 0.f};
        a = mfma(frag_row(K_, fo, 2 * hh + j, 0), qf0, a);
        c = mfma(frag_row(V_, fo, 2 * hh + j, 0), df0, c);
        a = mfma(frag_row(K_, fo, 2 * hh + j, 1), qf1, a);
        c = mfma(frag_row(V_, fo, 2 * hh + j, 1), df1, c);
        s[j] = a;
        dp[j] = c;
      }
      auto body = [&](auto FULL) {
        constexpr bool F = decltype(FULL)::value;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int bb = 2 * hh + j;
          unsigned kp = 0xfu;
          if (DROP) kp = keep4_rows(hs, qgbase, k0 + arow(bb, g, 0), li & 3, thr);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float x = fmaf(s[j][r], sl2, -lse2);
            if (!F) {
              const int key = k0 + arow(bb, g, r);
              if (key >= kvl || (p.causal && key > qrow)) x = -INFINITY;
            }
            const float pr = ex2(x);
            if (DROP) {
              const float dpk = (kp & (1u << r)) ? dp[j][r] : 0.f;
              ds[j][r] = pr * fmaf(dpk, keep_scale, -dlt);
            } else {
              ds[j][r] = pr * (dp[j][r] - dlt);
            }
          }
        }
      };
      if (full) body(bconst<true>{});
      else body(bconst<false>{});
      const bf16x8 sf = pack2(ds[0], ds[1]);
#pragma unroll
      for (int db = 0; db < 4; ++db) acc[db] = mfma(frag_tr(K_, fo, 32 * hh, db * 16), sf, acc[db]);
    }
    // unconditional: past the end these stage clamped rows into the idle buffer, never read
    tile_store<NTH>(kr, Ks[(t + 1) & 1]);
    tile_store<NTH>(vr, Vs[(t + 1) & 1]);
    tile_load<NTH>(kr, Kb, p.k_rs, k0 + 2 * TILE, kvl);
    tile_load<NTH>(vr, Vb, p.v_rs, k0 + 2 * TILE, kvl);
    lds_bar();
  }
  if (qrow < p.Sq) {
    bf16* dQ = p.dq + b * p.dq_bs + (long long)qrow * p.dq_rs + h * D;
#pragma unroll
    for (int db = 0; db < 4; ++db) store_rowvec4(dQ + db * 16 + 4 * g, acc[db], p.scale);
  }
}

// =============================================================================== dK/dV pass
template <int NW, bool DROP>
__global__ __launch_bounds__(NW * 64, NW == 8 ? 4 : 2) void attn_bwd_dkv_kernel(AttnParams p) {
  constexpr int NTH = NW * 64, RB = 16 * NW;  // threads; key rows per block
  __shared__ __attribute__((aligned(16))) bf16 Qs[2][TILE * LS];
  __shared__ __attribute__((aligned(16))) bf16 dOs[2][TILE * LS];
  __shared__ __attribute__((aligned(16))) float lse_s[2][TILE];
  __shared__ __attribute__((aligned(16))) float dlt_s[2][TILE];
  const int l = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), g = l >> 4, li = l & 15;
  FragOffs fo;
  fo.init();
  const int b = blockIdx.z, h = blockIdx.y, k0 = blockIdx.x * RB;
  const int bh = b * p.H + h;
  const uint32_t hs = head_seed(p, bh);
  const bf16* Qb = p.q + b * p.q_bs + h * D;
  const bf16* Kb = p.k + b * p.k_bs + h * D;
  const bf16* Vb = p.v + b * p.v_bs + h * D;
  const bf16* dOb = p.dout + b * p.o_bs + h * D;
  const float* lseb = p.lse + (long long)bh * p.Sq;
  const float* dltb = p.delta + (long long)bh * p.Sq;
  const int kvl = p.kv_len ? min(p.kv_len[b], p.Sk) : p.Sk;
  const int krow = k0 + 16 * w + li;  // this lane's key
  const int qstart = p.causal ? (k0 / TILE) * TILE : 0;
  const int ntiles = k0 < kvl ? (p.Sq - qstart + TILE - 1) / TILE : 0;
  // row statistics of the staged query tile: thread i < TILE carries query q0 + i
  // (unconditional loads, clamped row; padded rows get lse = +inf -> P = 0, delta = 0 at the store)
  auto stat_load = [&](int q0, float& ls, float& dl) {
    const int qq = min(q0 + (int)(threadIdx.x & (TILE - 1)), p.Sq - 1);
    ls = lseb[qq];
    dl = dltb[qq];
  };
  auto stat_store = [&](int q0, int buf, float ls, float dl) {
    const bool ok = q0 + (int)threadIdx.x < p.Sq;
    lse_s[buf][threadIdx.x] = ok ? ls * LOG2E : INFINITY;
    dlt_s[buf][threadIdx.x] = ok ? dl : 0.f;
  };
  TileRegs qr, dr;
  float nls = 0.f, ndl = 0.f;
  tile_load<NTH>(qr, Qb, p.q_rs, qstart, p.Sq);
  tile_load<NTH>(dr, dOb, p.o_rs, qstart, p.Sq);
  stat_load(qstart, nls, ndl);
  const bf16x8 kf0 = frag_global(Kb, p.k_rs, krow, kvl, 0), kf1 = frag_global(Kb, p.k_rs, krow, kvl, 1);
  const bf16x8 vf0 = frag_global(Vb, p.v_rs, krow, kvl, 0), vf1 = frag_global(Vb, p.v_rs, krow, kvl, 1);
  const float sl2 = p.scale * LOG2E;
  const int thr = drop_thr(p.p_drop);
  const float keep_scale = DROP ? 256.f / (float)(256 - thr) : 1.f;
  f32x4 dk[4], dv[4];
#pragma unroll
  for (int db = 0; db < 4; ++db) { dk[db] = f32x4{0.f, 0.f, 0.f, 0.f}; dv[db] = f32x4{0.f, 0.f, 0.f, 0.f}; }
  tile_store<NTH>(qr, Qs[0]);
  tile_store<NTH>(dr, dOs[0]);
  if (threadIdx.x < TILE) stat_store(qstart, 0, nls, ndl);
  tile_load<NTH>(qr, Qb, p.q_rs, qstart + TILE, p.Sq);
  tile_load<NTH>(dr, dOb, p.o_rs, qstart + TILE, p.Sq);
  stat_load(qstart + TILE, nls, ndl);
  lds_bar();
  // wave-uniform: this wave's 16 keys all valid (padded query rows are handled by lse = +inf)
  const bool keys_ok = k0 + 16 * w + 15 < kvl;
  for (int t = 0; t < ntiles; ++t) {
    const int q0 = qstart + t * TILE;
    const int cur = t & 1;
    const bf16* Q_ = Qs[cur];
    const bf16* O_ = dOs[cur];
    const bool full = keys_ok && (!p.causal || k0 + 16 * w + 15 <= q0);
    // two 32-query halves: S/dP of blocks 2hh, 2hh+1 -> P, dS -> their dV / dK MFMAs (k-slots
    // 32hh..32hh+31); half the live score registers of a whole-tile pass
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      f32x4 s[2], dp[2], pp[2], ds[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        f32x4 a = f32x4{0.f, 0.f, 0.f, 0.f}, c = f32x4{0.f, 0.f, 0.f, 0.f};
        a = mfma(frag_row(Q_, fo, 2 * hh + j, 0), kf0, a);
        c = mfma(frag_row(O_, fo, 2 * hh + j, 0), vf0, c);
        a = mfma(frag_row(Q_, fo, 2 * hh + j, 1), kf1, a);
        c = mfma(frag_row(O_, fo, 2 * hh + j, 1), vf1, c);
        s[j] = a;
        dp[j] = c;
      }
      auto body = [&](auto FULL) {
        constexpr bool F = decltype(FULL)::value;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int bb = 2 * hh + j;
          const int rb = 32 * (bb >> 1) + 8 * g + 4 * (bb & 1);  // tile rows arow(bb, g, 0..3)
          const f32x4 L = *(const f32x4*)&lse_s[cur][rb];
          const f32x4 Dl = *(const f32x4*)&dlt_s[cur][rb];
          unsigned kp = 0xfu;
          if (DROP) kp = keep4_cols(hs, (q0 + rb) >> 2, p.Sk, krow, thr);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float x = fmaf(s[j][r], sl2, -L[r]);
            if (!F && (krow >= kvl || (p.causal && krow > q0 + rb + r))) x = -INFINITY;
            const float pr = ex2(x);
            if (DROP) {
              const bool keep = kp & (1u << r);
              pp[j][r] = keep ? pr : 0.f;  // dV is scaled by keep_scale once at the store
              ds[j][r] = pr * fmaf(keep ? dp[j][r] : 0.f, keep_scale, -Dl[r]);
            } else {
              pp[j][r] = pr;
              ds[j][r] = pr * (dp[j][r] - Dl[r]);
            }
          }
        }
      };
      if (full) body(bconst<true>{});
      else body(bconst<false>{});
      const bf16x8 pf = pack2(pp[0], pp[1]), sf = pack2(ds[0], ds[1]);
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        dv[db] = mfma(frag_tr(O_, fo, 32 * hh, db * 16), pf, dv[db]);
        dk[db] = mfma(frag_tr(Q_, fo, 32 * hh, db * 16), sf, dk[db]);
      }
    }
    // unconditional: past the end these stage clamped rows into the idle buffer, never read
    tile_store<NTH>(qr, Qs[cur ^ 1]);
    tile_store<NTH>(dr, dOs[cur ^ 1]);
    if (threadIdx.x < TILE) stat_store(q0 + TILE, cur ^ 1, nls, ndl);
    tile_load<NTH>(qr, Qb, p.q_rs, q0 + 2 * TILE, p.Sq);
    tile_load<NTH>(dr, dOb, p.o_rs, q0 + 2 * TILE, p.Sq);
    stat_load(q0 + 2 * TILE, nls, ndl);
    lds_bar();
  }
  if (krow < p.Sk) {
    bf16* dK = p.dk + b * p.dk_bs + (long long)krow * p.dk_rs + h * D;
    bf16* dV = p.dv + b * p.dv_bs + (long long)krow * p.dv_rs + h * D;
#pragma unroll
    for (int db = 0; db < 4; ++db) {
      store_rowvec4(dK + db * 16 + 4 * g, dk[db], p.scale);
      store_rowvec4(dV + db * 16 + 4 * g, dv[db], keep_scale);
    }
  }
}
}  // namespace

// Waves per block (16 query/key rows each): 8 (default) shares every K/V (Q/dO) tile load and
// barrier pair between 128 rows instead of 64 -- measured Transformer-big self-attention fwd
// 50.5 -> 43.2 us, bwd 141.8 -> 129.9 us, bit-identical output. TFK_ATTN_WAVES=4|8. (A 16-wave
// 256-row block measured 23.31 vs 23.42 ms on Transformer-big but slower on BERT's S=128, and the
// dK/dV kernel's 163 VGPRs do not fit 1024-thread blocks: not kept.)
static int g_attn_waves = 0;
static int attn_waves() {
  if (g_attn_waves == 0) {
    const char* e = getenv("TFK_ATTN_WAVES");
    g_attn_waves = (e && e[0] == '4') ? 4 : 8;
  }
  return g_attn_waves;
}

extern "C" {
void tfk_attn_set_waves(int w) { g_attn_waves = w == 8 ? 8 : 4; }
// shape: [B, H, Sq, Sk]; strides: [q_bs, q_rs, k_bs, k_rs, v_bs, v_rs, o_bs, o_rs]
int tfk_attn_fwd(const void* q, const void* k, const void* v, void* out, float* lse, const long long* shape,
                 const long long* strides, const int* kv_len, float scale, int causal, float p_drop,
                 unsigned long long seed, hipStream_t s) {
  AttnParams p{};
  p.q = (const bf16*)q; p.k = (const bf16*)k; p.v = (const bf16*)v; p.out = (bf16*)out; p.lse = lse;
  p.B = (int)shape[0]; p.H = (int)shape[1]; p.Sq = (int)shape[2]; p.Sk = (int)shape[3];
  p.q_bs = strides[0]; p.q_rs = (int)strides[1]; p.k_bs = strides[2]; p.k_rs = (int)strides[3];
  p.v_bs = strides[4]; p.v_rs = (int)strides[5]; p.o_bs = strides[6]; p.o_rs = (int)strides[7];
  p.kv_len = kv_len; p.scale = scale; p.causal = causal; p.p_drop = p_drop; p.seed = seed; p.seed_key = tfk_seed_key();
  const bool drop = p_drop > 0.f;
  const dim3 g8((p.Sq + 127) / 128, p.H, p.B), g4((p.Sq + 63) / 64, p.H, p.B);
  if (attn_waves() == 8) {
    if (drop) hipLaunchKernelGGL((attn_fwd_kernel<8, true>), g8, dim3(512), 0, s, p);
    else hipLaunchKernelGGL((attn_fwd_kernel<8, false>), g8, dim3(512), 0, s, p);
  } else {
    if (drop) hipLaunchKernelGGL((attn_fwd_kernel<4, true>), g4, dim3(256), 0, s, p);
    else hipLaunchKernelGGL((attn_fwd_kernel<4, false>), g4, dim3(256), 0, s, p);
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
// grads: dq/dk/dv with strides [dq_bs, dq_rs, dk_bs, dk_rs, dv_bs, dv_rs]; delta: [B*H*Sq] scratch
int tfk_attn_bwd(const void* q, const void* k, const void* v, const void* o, const void* dout, const float* lse,
                 float* delta, void* dq, void* dk, void* dv, const long long* shape, const long long* strides,
                 const long long* gstrides, const int* kv_len, float scale, int causal, float p_drop,
                 unsigned long long seed, hipStream_t s) {
  AttnParams p{};
  p.q = (const bf16*)q; p.k = (const bf16*)k; p.v = (const bf16*)v; p.o = (const bf16*)o; p.dout = (const bf16*)dout;
  p.lse = (float*)lse; p.delta = delta; p.dq = (bf16*)dq; p.dk = (bf16*)dk; p.dv = (bf16*)dv;
  p.B = (int)shape[0]; p.H = (int)shape[1]; p.Sq = (int)shape[2]; p.Sk = (int)shape[3];
  p.q_bs = strides[0]; p.q_rs = (int)strides[1]; p.k_bs = strides[2]; p.k_rs = (int)strides[3];
  p.v_bs = strides[4]; p.v_rs = (int)strides[5]; p.o_bs = strides[6]; p.o_rs = (int)strides[7];
  p.dq_bs = gstrides[0]; p.dq_rs = (int)gstrides[1]; p.dk_bs = gstrides[2]; p.dk_rs = (int)gstrides[3];
  p.dv_bs = gstrides[4]; p.dv_rs = (int)gstrides[5];
  p.kv_len = kv_len; p.scale = scale; p.causal = causal; p.p_drop = p_drop; p.seed = seed; p.seed_key = tfk_seed_key();
  // delta = rowsum(dO * O) is computed and stored by the dQ kernel's prologue
  const bool drop = p_drop > 0.f;
  const dim3 q8((p.Sq + 127) / 128, p.H, p.B), k8((p.Sk + 127) / 128, p.H, p.B);
  const dim3 q4((p.Sq + 63) / 64, p.H, p.B), k4((p.Sk + 63) / 64, p.H, p.B);
#define TFK_ATTN_BWD(NW_, DROP_, GQ, GK)                                                       \
  hipLaunchKernelGGL((attn_bwd_dq_kernel<NW_, DROP_>), GQ, dim3(NW_ * 64), 0, s, p);          \
  hipLaunchKernelGGL((attn_bwd_dkv_kernel<NW_, DROP_>), GK, dim3(NW_ * 64), 0, s, p);
  if (attn_waves() == 8) {
    if (drop) { TFK_ATTN_BWD(8, true, q8, k8) } else { TFK_ATTN_BWD(8, false, q8, k8) }
  } else {
    if (drop) { TFK_ATTN_BWD(4, true, q4, k4) } else { TFK_ATTN_BWD(4, false, q4, k4) }
  }
#undef TFK_ATTN_BWD
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
}
