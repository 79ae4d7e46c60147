// inflate_tok.h — Huffman pass of the batched BGZF inflate (k_inflate_tokens), gfx950.
//
// Replaces [htsjdk] BlockGunzipper.unzipBlock -> java.util.zip.Inflater (JDK zlib) on the BAM
// read path; the observable contract is zlib 1.2.11's as documented in inflate_dev.h (ONE
// inflate(Z_PARTIAL_FLUSH) call with avail_out = ISIZE; identical error conditions).
//
// One lane decodes one BGZF block (SIMT over 64 blocks per wave).  What makes a lane-per-
// block decoder slow on CDNA is not the bit arithmetic but memory waits: a per-lane refill
// that loads the next 16 compressed bytes when the lane runs dry puts an
// `s_waitcnt vmcnt(...)` on the critical path of EVERY loop iteration, because some lane of
// the 64 is always refilling and the wait is per wave.  Here the input moves in wave-uniform
// epochs instead:
//   * each lane holds 32 compressed bytes in two register banks plus a 64-bit bit buffer;
//   * every TOK_K iterations (the same iteration for every active lane) a lane merges
//     the 16-byte quad it requested at the previous epoch into a free bank and requests the
//     next one, so a load has a whole epoch to land before anything waits on it;
//   * a lane that would need more bits than its banks hold skips the iteration (stall) until
//     the next epoch, which only happens on runs of long, far matches.
// Output (TSink): literals at their final ubuf offsets, a 3-byte descriptor (len-3, dist-1)
// at the start of every match hole, one bitmap bit per match start (128-position windows
// written as 16-byte stores), a 16-byte register write-combine chunk for the bytes.
// k_resolve (resolve_dev.h) then fills the holes.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "inflate_dev.h"

namespace hbam {

#if defined(HBAM_PROF) && !defined(HBAM_PROF_NOSTAMP)
// Profiling build only: wave-level cycles per region of the Huffman pass (tools/prof_regions.py)
#define TOK_PT(i)                                   \
  do {                                              \
    const uint64_t t_ = __builtin_amdgcn_s_memtime(); \
    pt[i] += t_ - tq;                               \
    tq = t_;                                        \
  } while (0)
#define TOK_PC(i) (++pc[i])
#else
#define TOK_PT(i) \
  do {            \
  } while (0)
#define TOK_PC(i) (void)0
#endif

constexpr uint32_t TOK_K = 4;  // symbol-loop iterations per input epoch (power of two)


// The fast path (tok_fast_spec): up to two literals and a match per iteration, decoded first
// (both lit/len lookups before either LDS symbol read), then written as one packet
// (TSink::put): 66.4 -> 60.3 ms at 10 GB against the same decode with one sink call per token
// (profiles/r02/s2/ab_spec_10g.txt).
// stream bits one fast-path iteration may consume: 2 lit/len codes + length extra + distance
// code + distance extra = 15+15+5+15+13 = 63 (<= 64)
constexpr uint32_t TOK_FAST_BITS = 64u;
constexpr uint32_t TOK_LENS_LL = 32;    // lens scratch: lit/len code lengths at +32 ..
constexpr uint32_t TOK_LENS_D = 320;    //               distance code lengths at +320 (<= 30)
constexpr uint32_t TOK_LENS_END = 352;  // = LENS_SLOT (hbam_internal.h)

// ---- input: two register banks + one quad in flight ------------------------------------
typedef const __attribute__((address_space(1))) u32x4_t* gq_ptr;  // global (not flat) loads
__device__ __forceinline__ u32x4_t ein_load(const uint4* p) { return *(gq_ptr)p; }
struct EIn {
  const uint4* fp;    // quad held in t (merged at the next epoch); == fend when the fetch is done
  const uint4* fend;  // one past the last quad that holds stream bytes
  const uint4* safe;  // an address already read (target of the dummy load after the fetch)
  uint4 q0, q1;       // banks: stream dwords, ring positions 0..3 and 4..7
  u32x4_t t;          // quad requested at the last epoch
  uint32_t rd;        // next ring position to move into bb
  uint32_t nv;        // unread dwords in the banks (from rd)
  uint64_t bb;        // bit buffer, LSB first
  uint32_t bc;        // valid bits in bb
  uint32_t consumed;  // stream bits consumed
  uint32_t total;     // 8 * deflated bytes
};

// (component-wise selects: a select between two uint4 lvalues becomes a select between their
// addresses, which pins the whole reader in scratch)
__device__ __forceinline__ uint32_t ein_sel(const EIn& e, uint32_t i) {
  const bool h = (i & 4u) != 0u, z = (i & 2u) != 0u;
  const uint32_t x = h ? e.q1.x : e.q0.x, y = h ? e.q1.y : e.q0.y;
  const uint32_t zz = h ? e.q1.z : e.q0.z, w = h ? e.q1.w : e.q0.w;
  const uint32_t a = z ? zz : x, b = z ? w : y;
  return (i & 1u) ? b : a;
}
__device__ __forceinline__ void ein_init(EIn& e, const uint8_t* p, uint32_t nbytes) {
  const uintptr_t a = (uintptr_t)p & 15u;
  const uint4* base = (const uint4*)(p - a);
  e.fend = (const uint4*)(((uintptr_t)(p + nbytes) + 15u) & ~(uintptr_t)15u);
  e.safe = base;
  e.q0 = base[0];
  e.q1 = base[1];
  e.fp = base + 2;
  if (e.fp > e.fend) e.fp = e.fend;
  e.t = ein_load(e.fp < e.fend ? e.fp : e.safe);
  const uint32_t r = (uint32_t)(a >> 2);
  const uint32_t sh = 8u * (uint32_t)(a & 3u);
  e.bb = (uint64_t)(ein_sel(e, r) >> sh);
  e.bc = 32u - sh;
  e.rd = r + 1u;
  e.nv = 8u - e.rd;
  e.consumed = 0;
  e.total = nbytes * 8u;
}
// one dword from the banks into bb (the stall check guarantees the banks hold what is needed)
__device__ __forceinline__ void ein_refill(EIn& e) {
  if (e.bc <= 32u && e.nv != 0u) {
    e.bb |= (uint64_t)ein_sel(e, e.rd) << e.bc;
    e.bc += 32u;
    e.rd = (e.rd + 1u) & 7u;
    --e.nv;
  }
}
// the same without a branch (the fast path: a branch around it costs every iteration the exec-mask
// bookkeeping, since some lane of 64 nearly always needs the dword).  With the branchless length /
// distance bases below: Huffman 33.9 -> 32.1 ms at 5 GB, same output
// (profiles/r05/ab/huffman_branchless_refill_bases_5g.txt)
__device__ __forceinline__ void ein_refill_sel(EIn& e) {
  const bool need = e.bc <= 32u && e.nv != 0u;
  const uint64_t add = (uint64_t)ein_sel(e, e.rd) << (e.bc & 63u);
  e.bb |= need ? add : 0ull;
  e.bc += need ? 32u : 0u;
  e.rd = need ? ((e.rd + 1u) & 7u) : e.rd;
  e.nv -= need ? 1u : 0u;
}
// length / distance bases without branches (DEFLATE tables as arithmetic; RFC 1951 3.2.5)
// (one formula for every code, the exceptions as constant selects: written as a select between
// two computed arms, the compiler turned the length base back into a branch)
__device__ __forceinline__ void length_base_sel(uint32_t sym, uint32_t& base, uint32_t& extra) {
  const uint32_t i = sym - 257u;  // [0, 28]
  const uint32_t ex = ((i > 4u ? i : 4u) - 4u) >> 2;  // 0 for codes 257-264
  const uint32_t b = ((4u + (i & 3u)) << ex) + 3u - (i < 4u ? 4u : 0u);
  extra = i < 28u ? ex : 0u;
  base = i < 28u ? b : 258u;
}
__device__ __forceinline__ void dist_base_sel(uint32_t d, uint32_t& base, uint32_t& extra) {
  const uint32_t ex = ((d > 2u ? d : 2u) >> 1) - 1u;  // 0 for codes 0-3
  extra = ex;
  base = ((2u + (d & 1u)) << ex) + 1u - (d < 2u ? 2u : 0u);
}
// epoch boundary: merge the quad in flight into the free bank, request the next one
__device__ __forceinline__ void ein_epoch_merge(EIn& e) {
  if (e.fp < e.fend && e.nv <= 4u) {
    const bool hi = (((e.rd + e.nv) & 7u) >> 2) != 0u;
    const u32x4_t t = e.t;
    e.q0.x = hi ? e.q0.x : t[0];
    e.q0.y = hi ? e.q0.y : t[1];
    e.q0.z = hi ? e.q0.z : t[2];
    e.q0.w = hi ? e.q0.w : t[3];
    e.q1.x = hi ? t[0] : e.q1.x;
    e.q1.y = hi ? t[1] : e.q1.y;
    e.q1.z = hi ? t[2] : e.q1.z;
    e.q1.w = hi ? t[3] : e.q1.w;
    e.nv += 4u;
    ++e.fp;
  }
}
__device__ __forceinline__ void ein_epoch_load(EIn& e) { e.t = ein_load(e.fp < e.fend ? e.fp : e.safe); }
__device__ __forceinline__ void ein_epoch(EIn& e) {
  ein_epoch_merge(e);
  ein_epoch_load(e);
}
// bits the lane can use without another epoch
__device__ __forceinline__ bool ein_short(const EIn& e, uint32_t need) {
  return e.bc + 32u * e.nv < need && e.fp < e.fend;
}
// synchronous top-up (header phase): epochs until `need` bits are buffered or the fetch is done
__device__ __forceinline__ void ein_ensure(EIn& e, uint32_t need) {
  while (ein_short(e, need)) ein_epoch(e);
  ein_refill(e);
  ein_refill(e);
}
__device__ __forceinline__ uint32_t ein_avail(const EIn& e) { return e.total - e.consumed; }
__device__ __forceinline__ uint32_t ein_peek(const EIn& e, uint32_t n) {
  return (uint32_t)e.bb & ((1u << n) - 1u);
}
__device__ __forceinline__ void ein_drop(EIn& e, uint32_t n) {
  e.bb >>= n;
  e.bc -= n;
  e.consumed += n;
}
__device__ __forceinline__ uint32_t ein_rev15(const EIn& e) {
  return __builtin_bitreverse32((uint32_t)e.bb) >> 17;
}

// ---- packed canonical decode tables (symbol loop) ---------------------------------------
// The lookup is the loop's largest VALU cost: 14 compares of the 15-bit code against the
// per-length limits, each feeding a length count, an index offset and (lit/len) the symbol's
// bit 8.  Pairs of limits in 16-bit halves let one v_pk_sub_u16 (clamp) + v_pk_min_u16 form
// two compare results as 0/1 halves and v_pk_mad_u16 fold them into the offsets, about half
// the instructions of the 32-bit chain.  Offsets are kept as 16-bit deltas: the sums are exact
// mod 2^16 and every valid index is < 288.
typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));
typedef int16_t i16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u16x2 as_u16x2(uint32_t x) { return __builtin_bit_cast(u16x2, x); }
__device__ __forceinline__ uint32_t as_u32(u16x2 x) { return __builtin_bit_cast(uint32_t, x); }
__device__ __forceinline__ uint32_t pk2(uint32_t lo, uint32_t hi) { return (lo & 0xffffu) | hi << 16; }
struct HuffP {
  uint32_t lim[7];  // (lim[2j], lim[2j+1]) as u16 halves
  uint32_t dof[7];  // (doff[2j+1], doff[2j+2])
  uint32_t dhl[7];  // lit/len: (hlim[2j+1] - hlim[2j], hlim[2j+2] - hlim[2j+1])
  uint32_t lim14;   // v < lim14 <=> v starts a valid code
  uint32_t o0;      // doff[0]
  uint32_t t0;      // hlim[0]
};
__device__ __forceinline__ void huffp_make(const Huff& h, HuffP& p) {
#pragma unroll
  for (int j = 0; j < 7; ++j) {
    p.lim[j] = pk2(h.lim[2 * j], h.lim[2 * j + 1]);
    p.dof[j] = pk2((uint32_t)h.doff[2 * j + 1], (uint32_t)h.doff[2 * j + 2]);
    p.dhl[j] = pk2(h.hlim[2 * j + 1] - h.hlim[2 * j], h.hlim[2 * j + 2] - h.hlim[2 * j + 1]);
  }
  p.lim14 = h.lim[14];
  p.o0 = (uint32_t)h.doff[0];
  p.t0 = h.hlim[0];
}
// code length / symbol index (/ bit 8 of a lit/len symbol) of a left-justified 15-bit value;
// false: no code starts with v
// Per pair j (inline VOP3P, one asm statement per group of pairs: written as vector C, LLVM
// turns min(sub_sat) back into per-half compares and selects, and separate asm statements
// each cost a hazard s_nop):
//   g  = min(sat(v+1 - lim_j), 1)   the two "v >= lim" bits as 0/1 halves
//   sl += g;  so += g * dof_j;  st += g * dhl_j
// v_dot2_u32_u16 folds both halves into one u32 accumulator per pair, so the sums need no
// final (x & 0xffff) + (x >> 16) step (offsets stay exact mod 2^16: results are masked)
#define HBAM_PK_PAIR(LIM, DOF, DHL)                 \
  "v_pk_sub_u16 %[g], %[vv], " LIM " clamp\n\t"     \
  "v_pk_min_u16 %[g], %[g], %[one]\n\t"              \
  "v_dot2_u32_u16 %[sl], %[g], %[one], %[sl]\n\t"    \
  "v_dot2_u32_u16 %[so], %[g], " DOF ", %[so]\n\t"   \
  "v_dot2_u32_u16 %[st], %[g], " DHL ", %[st]\n\t"
#define HBAM_PK_PAIR_NT(LIM, DOF)                   \
  "v_pk_sub_u16 %[g], %[vv], " LIM " clamp\n\t"     \
  "v_pk_min_u16 %[g], %[g], %[one]\n\t"              \
  "v_dot2_u32_u16 %[sl], %[g], %[one], %[sl]\n\t"    \
  "v_dot2_u32_u16 %[so], %[g], " DOF ", %[so]\n\t"
// Two pairs at a time with two compare registers: the sub -> min -> dot2 chain of one pair has the
// other pair's instructions between its links instead of stalling on them (A/B at 5 GB: Huffman
// 34.1 -> 33.8 ms, same output; profiles/r05/ab/pools_windows_tok_ilv_5g.txt).
#define HBAM_PK2_PAIR(LA, DA, TA, LB, DB, TB)          \
  "v_pk_sub_u16 %[g], %[vv], " LA " clamp\n\t"        \
  "v_pk_sub_u16 %[h], %[vv], " LB " clamp\n\t"        \
  "v_pk_min_u16 %[g], %[g], %[one]\n\t"               \
  "v_pk_min_u16 %[h], %[h], %[one]\n\t"               \
  "v_dot2_u32_u16 %[sl], %[g], %[one], %[sl]\n\t"     \
  "v_dot2_u32_u16 %[so], %[g], " DA ", %[so]\n\t"     \
  "v_dot2_u32_u16 %[st], %[g], " TA ", %[st]\n\t"     \
  "v_dot2_u32_u16 %[sl], %[h], %[one], %[sl]\n\t"     \
  "v_dot2_u32_u16 %[so], %[h], " DB ", %[so]\n\t"     \
  "v_dot2_u32_u16 %[st], %[h], " TB ", %[st]\n\t"
#define HBAM_PK2_PAIR_NT(LA, DA, LB, DB)               \
  "v_pk_sub_u16 %[g], %[vv], " LA " clamp\n\t"        \
  "v_pk_sub_u16 %[h], %[vv], " LB " clamp\n\t"        \
  "v_pk_min_u16 %[g], %[g], %[one]\n\t"               \
  "v_pk_min_u16 %[h], %[h], %[one]\n\t"               \
  "v_dot2_u32_u16 %[sl], %[g], %[one], %[sl]\n\t"     \
  "v_dot2_u32_u16 %[so], %[g], " DA ", %[so]\n\t"     \
  "v_dot2_u32_u16 %[sl], %[h], %[one], %[sl]\n\t"     \
  "v_dot2_u32_u16 %[so], %[h], " DB ", %[so]\n\t"
template <bool HI>
__device__ __forceinline__ bool huffp_lookup(const HuffP& h, uint32_t v, uint32_t& L, uint32_t& idx,
                                             uint32_t& hi) {
  const uint32_t vv = (v + 1u) * 0x10001u;  // v + 1 <= 32768 in both halves
  const uint32_t one = 0x10001u;
  uint32_t sl = 0, so = 0, st = 0, g;
  uint32_t g2;
  if (HI) {
    asm(HBAM_PK2_PAIR("%[l0]", "%[d0]", "%[t0]", "%[l1]", "%[d1]", "%[t1]")
        HBAM_PK2_PAIR("%[l2]", "%[d2]", "%[t2]", "%[l3]", "%[d3]", "%[t3]")
        : [sl] "+v"(sl), [so] "+v"(so), [st] "+v"(st), [g] "=&v"(g), [h] "=&v"(g2)
        : [vv] "v"(vv), [one] "v"(one), [l0] "v"(h.lim[0]), [l1] "v"(h.lim[1]), [l2] "v"(h.lim[2]),
          [l3] "v"(h.lim[3]), [d0] "v"(h.dof[0]), [d1] "v"(h.dof[1]), [d2] "v"(h.dof[2]),
          [d3] "v"(h.dof[3]), [t0] "v"(h.dhl[0]), [t1] "v"(h.dhl[1]), [t2] "v"(h.dhl[2]),
          [t3] "v"(h.dhl[3]));
    asm(HBAM_PK2_PAIR("%[l4]", "%[d4]", "%[t4]", "%[l5]", "%[d5]", "%[t5]")
        HBAM_PK_PAIR("%[l6]", "%[d6]", "%[t6]")
        : [sl] "+v"(sl), [so] "+v"(so), [st] "+v"(st), [g] "=&v"(g), [h] "=&v"(g2)
        : [vv] "v"(vv), [one] "v"(one), [l4] "v"(h.lim[4]), [l5] "v"(h.lim[5]), [l6] "v"(h.lim[6]),
          [d4] "v"(h.dof[4]), [d5] "v"(h.dof[5]), [d6] "v"(h.dof[6]), [t4] "v"(h.dhl[4]),
          [t5] "v"(h.dhl[5]), [t6] "v"(h.dhl[6]));
  } else {
    asm(HBAM_PK2_PAIR_NT("%[l0]", "%[d0]", "%[l1]", "%[d1]") HBAM_PK2_PAIR_NT("%[l2]", "%[d2]", "%[l3]", "%[d3]")
        HBAM_PK2_PAIR_NT("%[l4]", "%[d4]", "%[l5]", "%[d5]") HBAM_PK_PAIR_NT("%[l6]", "%[d6]")
        : [sl] "+v"(sl), [so] "+v"(so), [g] "=&v"(g), [h] "=&v"(g2)
        : [vv] "v"(vv), [one] "v"(one), [l0] "v"(h.lim[0]), [l1] "v"(h.lim[1]), [l2] "v"(h.lim[2]),
          [l3] "v"(h.lim[3]), [l4] "v"(h.lim[4]), [l5] "v"(h.lim[5]), [l6] "v"(h.lim[6]),
          [d0] "v"(h.dof[0]), [d1] "v"(h.dof[1]), [d2] "v"(h.dof[2]), [d3] "v"(h.dof[3]),
          [d4] "v"(h.dof[4]), [d5] "v"(h.dof[5]), [d6] "v"(h.dof[6]));
  }
  const uint32_t l = 1u + sl;
  L = l;
  idx = (h.o0 + so + (v >> (15u - l))) & 0xffffu;
  if (HI) hi = v >= ((h.t0 + st) & 0xffffu) ? 256u : 0u;
  return v < h.lim14;
}

// ---- output ------------------------------------------------------------------------------
struct TSink {
  uint8_t* cbase;   // 16-aligned address of chunk 0 (the chunk holding the block's first byte)
  uint32_t soff;    // block start inside chunk 0
  uint32_t iend;    // soff + isize
  uint32_t curc;    // chunk held in lo/hi (0 at the start: the block's first byte is in chunk 0)
  uint64_t lo, hi;
  uint32_t* bm;     // match-start bitmap of the block (BITMAP_WORDS words)
  uint32_t bwin;    // 128-position window held in wl (positions 0-63) / wh (64-127)
  uint32_t nwin;    // windows covering the block
  uint64_t wl, wh;
  uint32_t* tail;   // [0] = op | n<<16 | 1<<31 for a final match shorter than 3 bytes, [1] = dist
  uint32_t t0, t1;  // tail[0..1], stored by finish() (a store behind a branch in the loop cost
                    // every iteration its exec-mask bookkeeping; with the unconditional chunk 0
                    // and the 64-bit bitmap words: Huffman 32.5 -> 31.0 ms at 5 GB, same output,
                    // profiles/r05/ab/huffman_sink_tail_mark_5g.txt)
  uint8_t* edge;    // 32 B: the block's partial first / last 16-byte chunk (k_edge_merge)

  __device__ __forceinline__ void init(uint8_t* ubuf, uint64_t start, uint32_t isize, uint32_t* bmp,
                                       uint32_t* tl, uint8_t* eg) {
    edge = eg;
    cbase = ubuf + (start & ~15ull);
    soff = (uint32_t)(start & 15u);
    iend = soff + isize;
    curc = 0;  // (a flush before any output writes zeros to the block's own chunk 0 / edge slot)
    lo = hi = 0;
    bm = bmp;
    bwin = 0;
    nwin = (isize + 127u) >> 7;
    wl = wh = 0;
    tail = tl;
    t0 = t1 = 0;
  }
  __device__ __forceinline__ void flush() {
    const uint32_t r0 = curc << 4;
    // A chunk shared with a neighbouring block (the block's first chunk when it does not
    // start 16-aligned, its last when it does not end so) goes to the block's edge slot
    // instead, whole; k_edge_merge writes this block's bytes of it afterwards.  So every flush
    // is one 16-byte store and the loop carries no byte-store fallback.
    const bool full = r0 >= soff && r0 + 16u <= iend;
    uint8_t* dst = full ? cbase + r0 : edge + (r0 < soff ? 0u : 16u);
    st_out((uint4*)dst, make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)));
  }
  __device__ __forceinline__ void chunk(uint32_t c) {
    if (c != curc) {
      flush();
      curc = c;
      lo = 0;
      hi = 0;
    }
  }
  __device__ __forceinline__ void win_store() {
    st_out((uint4*)(bm + 4u * bwin),
           make_uint4((uint32_t)wl, (uint32_t)(wl >> 32), (uint32_t)wh, (uint32_t)(wh >> 32)));
  }
  __device__ __forceinline__ void mark(uint32_t op) { mark_if(true, op); }
  // the match-start bit of op when em: the bit as selects, only the window store behind a branch
  __device__ __forceinline__ void mark_if(bool em, uint32_t op) {
    const uint32_t w = op >> 7;
    if (em && bwin < w) {
      win_store();
      wl = wh = 0;
      ++bwin;
      while (bwin < w) {  // a match longer than the window: zero windows
        win_store();
        ++bwin;
      }
    }
    const uint32_t i = op & 127u;
    const uint64_t m = 1ull << (i & 63u);  // one 64-bit shift and two selects (was four compares)
    wl |= (em && i < 64u) ? m : 0ull;
    wh |= (em && i >= 64u) ? m : 0ull;
  }
  __device__ __forceinline__ void literal(uint32_t op, uint32_t b) {
    const uint32_t r = soff + op;
    chunk(r >> 4);
    const uint64_t v = (uint64_t)(b & 0xffu) << ((r & 7u) << 3);
    if (r & 8u) hi |= v;
    else lo |= v;
  }
  __device__ __forceinline__ void match(uint32_t op, uint32_t n, uint32_t dist) {
    if (n < 3u) {  // the output filled up inside the match: last token of the block
      t0 = op | n << 16 | 0x80000000u;
      t1 = dist;
      return;
    }
    const uint64_t d = (uint64_t)((n - 3u) | (dist - 1u) << 8);  // 3 bytes
    const uint32_t r = soff + op;
    const uint32_t c = r >> 4, k = r & 15u;
    chunk(c);
    if (k < 8u) {
      lo |= d << (8u * k);
      if (k > 5u) hi |= d >> (64u - 8u * k);
    } else {
      hi |= d << (8u * (k - 8u));  // bytes past the chunk (k >= 14) fall off here ...
    }
    if (k >= 14u) {  // ... and start the next chunk
      const uint64_t spill = d >> (8u * (16u - k));
      flush();
      curc = c + 1u;
      lo = spill;
      hi = 0;
    }
    mark(op);
  }
  // chunk switch as a predicated step: only the flush (a store) sits behind a branch
  __device__ __forceinline__ void switch_if(bool sw, uint32_t c) {
    if (sw) flush();
    curc = sw ? c : curc;
    lo = sw ? 0ull : lo;
    hi = sw ? 0ull : hi;
  }
  // One iteration's output as one packet: nb (<= 5) bytes P (LSB first) at ubuf position
  // soff + op: up to two literals and a 3-byte match descriptor, always contiguous, so one
  // chunk switch and at most one spill into the next chunk (tok_fast_spec).
  __device__ __forceinline__ void put(uint32_t op, uint64_t P, uint32_t nb) {
    const bool any = nb != 0u;
    const uint32_t r = soff + op;
    const uint32_t c = r >> 4, k = r & 15u;
    switch_if(any && c != curc, c);
    // shift amounts below 64 in every select arm (P < 2^40: at most 5 bytes)
    const uint32_t kl = k < 8u ? k : 0u, kh = k < 8u ? 0u : k - 8u;
    const uint32_t kr = (k > 1u && k < 8u) ? 64u - 8u * k : 8u;
    lo |= k < 8u ? P << (8u * kl) : 0ull;
    hi |= (k > 1u && k < 8u) ? P >> kr : 0ull;
    hi |= k < 8u ? 0ull : P << (8u * kh);
    const bool sp = any && k + nb > 16u;
    if (sp) flush();
    const uint64_t spill = P >> (8u * (16u - (k >= 10u ? k : 10u)));
    curc = sp ? c + 1u : curc;
    lo = sp ? spill : lo;
    hi = sp ? 0ull : hi;
  }
  __device__ __forceinline__ void finish() {
    flush();
    tail[0] = t0;
    tail[1] = t1;
    while (bwin < nwin) {
      win_store();
      wl = wh = 0;
      ++bwin;
    }
  }
};

// ---- canonical tables from code lengths in global scratch ---------------------------------
// lens: 16-aligned global bytes (n of them); kind 0 = code lengths, 1 = lit/len, 2 = distances.
// The lengths are read 16 at a time, the next quad requested before the current one is
// processed (one wait per 16 symbols instead of one per symbol).
__device__ __forceinline__ uint32_t quad_byte(const uint4& q, uint32_t j) {  // j compile-time
  const uint32_t w = j < 4 ? q.x : j < 8 ? q.y : j < 12 ? q.z : q.w;
  return (w >> (8u * (j & 3u))) & 0xffu;
}
// Out of line: called once per DEFLATE block, and inlining its unrolled counters into the
// kernel pushes the symbol loop's state into scratch.
__device__ __attribute__((noinline)) bool tok_build(const uint8_t* __restrict__ lens, int n,
                                                    uint8_t* __restrict__ syms, Huff& h, int kind) {
  typedef uint8_t SymT;
  const uint4* lq = (const uint4*)lens;
  const int nq = (n + 15) >> 4;
  uint32_t cnt[16], nhi[16];
#pragma unroll
  for (int L = 0; L < 16; ++L) cnt[L] = nhi[L] = 0;
  uint4 qn = lq[0];
  for (int k = 0; k < nq; ++k) {
    const uint4 q = qn;
    if (k + 1 < nq) qn = lq[k + 1];
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j) {
      const int s = 16 * k + (int)j;
      const uint32_t len = s < n ? quad_byte(q, j) : 0u;
      const uint32_t hb = (kind == 1 && s >= 256) ? 1u : 0u;
#pragma unroll
      for (int L = 1; L < 16; ++L) {
        cnt[L] += (len == (uint32_t)L) ? 1u : 0u;
        nhi[L] += (len == (uint32_t)L) ? hb : 0u;
      }
    }
  }
  uint32_t maxl = 0;
#pragma unroll
  for (int L = 1; L < 16; ++L) maxl = cnt[L] ? (uint32_t)L : maxl;
  h.empty = (maxl == 0);
  if (maxl != 0) {
    int32_t left = 1;
    bool over = false;
#pragma unroll
    for (int L = 1; L < 16; ++L) {
      left = 2 * left - (int32_t)cnt[L];
      over |= left < 0;
    }
    if (over) return false;
    if (left > 0 && (kind == 0 || maxl != 1)) return false;  // incomplete set
  }
  uint32_t code = 0, base = 0;
  uint32_t next[16];
  int32_t prev_off = 0;
#pragma unroll
  for (int L = 1; L < 16; ++L) {
    h.lim[L - 1] = (code + cnt[L]) << (15 - L);
    h.hlim[L - 1] = (code + cnt[L] - nhi[L]) << (15 - L);
    const int32_t off = (int32_t)base - (int32_t)code;
    h.doff[L - 1] = off - prev_off;
    prev_off = off;
    next[L] = base;
    base += cnt[L];
    code = (code + cnt[L]) << 1;
  }
  if (maxl == 0) {
#pragma unroll
    for (int L = 0; L < 15; ++L) h.lim[L] = h.hlim[L] = 0;
  }
  qn = lq[0];
  for (int k = 0; k < nq; ++k) {
    const uint4 q = qn;
    if (k + 1 < nq) qn = lq[k + 1];
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j) {
      const int s = 16 * k + (int)j;
      const uint32_t len = s < n ? quad_byte(q, j) : 0u;
      if (len) {
        uint32_t pos = 0;
#pragma unroll
        for (int L = 1; L < 16; ++L) {
          const bool eq = (len == (uint32_t)L);
          pos = eq ? next[L] : pos;
          next[L] += eq ? 1u : 0u;
        }
        syms[pos] = (SymT)s;
      }
    }
  }
  return true;
}

// One iteration of the symbol loop with >= 64 stream bits left: two lit/len codes + length
// extra + distance code + distance extra (15+15+5+15+13) fit, so zlib's end-of-input outcomes
// cannot occur and after one refill (>= 33 bits in bb) none is checked.  A literal is followed
// by a second lit/len decode in the same iteration (the wave pays for the match path once per
// iteration either way, and most symbols are literals).  Every lane runs the whole iteration
// and flags say which of its results count (SIMT runs the union of the paths anyway); the
// first exit code a lane meets wins, as zlib's early returns.  Both lit/len lookups run before
// either symbol read (the second on the bits after the first code, whether or not it turns out
// to be used), so the two LDS reads are in flight together; the iteration's bytes (up to two
// literals and a match descriptor, contiguous) go to the sink as one packet.
// Returns 0 next, 1 end of block, 2 output full (zlib stops), 3 data error.
// An iteration's packet and match mark are handed to the next iteration (TPend), which writes
// them while its own symbol reads are in flight (the packet after the two lit/len reads, the mark
// after the distance read); whether a symbol is a literal comes from the code's bit 8 (huffp_lookup's
// hi), not from the LDS byte.  Each LDS round trip costs a wave ~100 cycles of its ~3.3 k-cycle
// iteration (a probe with every symbol read doubled into two dependent reads: Huffman 30.4 ->
// 32.5 ms at 5 GB); with the writes in the shadow of the reads: 30.95 / 31.15 -> 30.10 / 30.10 ms,
// same output (profiles/r06/ab/huffman_deferred_packet_5g.txt).
struct TPend {
  uint64_t P;
  uint32_t op1, nb, opm;
  bool em;
  __device__ __forceinline__ void clear() {
    P = 0;
    op1 = nb = opm = 0;
    em = false;
  }
  __device__ __forceinline__ void flush(TSink& sink) {
    sink.put(op1, P, nb);
    sink.mark_if(em, opm);
    P = 0;  // put ORs P in whatever nb says
    nb = 0;
    em = false;
  }
};
__device__ __forceinline__ uint32_t tok_fast_spec(EIn& in, const HuffP& hl, const HuffP& hd,
                                                  const uint8_t* __restrict__ syms_ll,
                                                  const uint8_t* __restrict__ syms_d, TSink& sink,
                                                  uint32_t& op, uint32_t isize, TPend& pd) {
  ein_refill_sel(in);
  uint32_t L1, idx1, hi1 = 0, L2, idx2, hi2 = 0;
  const bool ok1 = huffp_lookup<true>(hl, ein_rev15(in), L1, idx1, hi1);
  const uint32_t l1 = ok1 ? L1 : 0u;
  const uint32_t v2 = __builtin_bitreverse32((uint32_t)(in.bb >> l1)) >> 17;
  const bool ok2 = huffp_lookup<true>(hl, v2, L2, idx2, hi2);
  const uint32_t sym1 = (uint32_t)syms_ll[ok1 ? idx1 : 0u] | hi1;
  const uint32_t sym2 = (uint32_t)syms_ll[ok2 ? idx2 : 0u] | hi2;
  sink.put(pd.op1, pd.P, pd.nb);  // the previous iteration's packet
  uint32_t ex = ok1 ? 0u : 3u;
  ein_drop(in, l1);
  const bool lit1 = ok1 && hi1 == 0u;
  ex = (ex == 0u && lit1 && op == isize) ? 2u : ex;
  const bool emit1 = ex == 0u && lit1;
  const uint32_t op1 = op;
  op += emit1 ? 1u : 0u;
  ex = (emit1 && !ok2) ? 3u : ex;
  ein_drop(in, (emit1 && ok2) ? L2 : 0u);
  const bool lit2 = emit1 && ok2 && hi2 == 0u;
  ex = (ex == 0u && lit2 && op == isize) ? 2u : ex;
  const bool emit2 = ex == 0u && lit2;
  op += emit2 ? 1u : 0u;
  const uint32_t m = emit1 ? sym2 : sym1;
  const bool ism = ex == 0u && !emit2 && !lit2;
  ex = (ism && m == 256u) ? 1u : ex;
  ex = (ism && m > 285u) ? 3u : ex;
  const bool dom = ism && m > 256u && m <= 285u;
  uint32_t lbase, lext;
  length_base_sel(dom ? m : 257u, lbase, lext);
  ein_refill_sel(in);
  lext = dom ? lext : 0u;
  const uint32_t mlen = lbase + ein_peek(in, lext);
  ein_drop(in, lext);
  uint32_t L, idx, dh;
  const bool okd = huffp_lookup<false>(hd, ein_rev15(in), L, idx, dh);
  const uint32_t dsym = syms_d[okd ? idx : 0u];
  sink.mark_if(pd.em, pd.opm);  // the previous iteration's match mark
  ex = (dom && !okd) ? 3u : ex;
  ein_drop(in, (dom && okd) ? L : 0u);
  ex = (dom && okd && dsym > 29u) ? 3u : ex;
  const bool dom2 = dom && ex == 0u;
  uint32_t dbase, dext;
  dist_base_sel(dom2 ? dsym : 0u, dbase, dext);
  dext = dom2 ? dext : 0u;
  const uint32_t dist = dbase + ein_peek(in, dext);
  ein_drop(in, dext);
  ex = (dom2 && op == isize) ? 2u : ex;
  ex = (dom2 && ex == 0u && dist > op) ? 3u : ex;
  const bool domatch = dom2 && ex == 0u;
  uint32_t n = isize - op;
  n = mlen < n ? mlen : n;
  const bool last = domatch && n < 3u;  // the output filled up inside the match: last token
  sink.t0 = last ? (op | n << 16 | 0x80000000u) : sink.t0;
  sink.t1 = last ? dist : sink.t1;
  const bool em = domatch && n >= 3u;
  uint64_t P = emit1 ? (uint64_t)(sym1 & 0xffu) : 0ull;
  P |= emit2 ? (uint64_t)(sym2 & 0xffu) << 8 : 0ull;
  const uint32_t nl = (emit1 ? 1u : 0u) + (emit2 ? 1u : 0u);
  P |= em ? (uint64_t)((n - 3u) | (dist - 1u) << 8) << (8u * nl) : 0ull;
  pd.op1 = op1;
  pd.P = P;
  pd.nb = nl + (em ? 3u : 0u);
  pd.em = em;
  pd.opm = op;
  op += domatch ? n : 0u;
  ex = (domatch && n < mlen) ? 2u : ex;
  return ex;
}
// One symbol with every zlib outcome checked (the stream's last 64 bits).
__device__ __forceinline__ uint32_t tok_careful(EIn& in, const HuffP& hl, const HuffP& hd,
                                                const uint8_t* __restrict__ syms_ll,
                                                const uint8_t* __restrict__ syms_d, TSink& sink,
                                                uint32_t& op, uint32_t isize) {
  ein_refill(in);
  uint32_t L, idx, hi = 0;
  if (!huffp_lookup<true>(hl, ein_rev15(in), L, idx, hi)) return ein_avail(in) >= 1u ? 3u : 2u;
  if (L > ein_avail(in)) return 2u;
  const uint32_t sym = (uint32_t)syms_ll[idx] | hi;
  ein_drop(in, L);
  if (sym < 256u) {
    if (op == isize) return 2u;
    sink.literal(op++, sym);
    return 0u;
  }
  if (sym == 256u) return 1u;
  if (sym > 285u) return 3u;
  uint32_t lbase, lext;
  length_base(sym, lbase, lext);
  if (lext > ein_avail(in)) return 2u;
  const uint32_t mlen = lbase + ein_peek(in, lext);
  ein_drop(in, lext);
  ein_refill(in);
  uint32_t dh;
  if (!huffp_lookup<false>(hd, ein_rev15(in), L, idx, dh)) return ein_avail(in) >= 1u ? 3u : 2u;
  if (L > ein_avail(in)) return 2u;
  const uint32_t dsym = syms_d[idx];
  ein_drop(in, L);
  if (dsym > 29u) return 3u;
  uint32_t dbase, dext;
  dist_base(dsym, dbase, dext);
  if (dext > ein_avail(in)) return 2u;
  const uint32_t dist = dbase + ein_peek(in, dext);
  ein_drop(in, dext);
  if (op == isize) return 2u;
  if (dist > op) return 3u;
  uint32_t n = isize - op;
  n = mlen < n ? mlen : n;
  sink.match(op, n, dist);
  op += n;
  return n < mlen ? 2u : 0u;
}

// Inflate one raw DEFLATE stream (cdata, nbytes) to exactly isize bytes into the token sink.
// syms_ll: 288 u8 LDS slots (symbol & 255; bit 8 from Huff.hlim); syms_d: 32 u8 LDS slots;
// lens: LENS_SLOT bytes of 16-aligned global scratch.  Returns INF_OK / INF_SHORT / INF_DATA.
__device__ __forceinline__ int32_t inflate_tokens_block(const uint8_t* __restrict__ cdata, uint32_t nbytes,
                                        uint32_t isize, uint8_t* __restrict__ syms_ll,
                                        uint8_t* __restrict__ syms_d, uint8_t* __restrict__ lens,
                                        TSink& sink, uint32_t* produced
#ifdef HBAM_PROF
                                        , uint64_t* pt, uint64_t* pc
#endif
                                        ) {
#ifdef HBAM_PROF
  uint64_t tq = __builtin_amdgcn_s_memtime();
#endif
  EIn in;
  ein_init(in, cdata, nbytes);
  uint32_t op = 0;
  HuffP hl, hd;
  bool last = false;
  int32_t rc = INF_OK;
  uint32_t it = 0;  // iteration counter shared by the lanes of a phase (epoch clock)
  for (;;) {
    if (last) break;  // stream end
    ein_ensure(in, 64);
    if (ein_avail(in) < 3u) goto leave;
    last = (in.bb & 1u) != 0;
    {
      const uint32_t type = (uint32_t)(in.bb >> 1) & 3u;
      ein_drop(in, 3);
      if (type == 0u) {
        // stored: byte align, LEN/NLEN, then LEN literal bytes
        const uint32_t pad = (8u - (in.consumed & 7u)) & 7u;
        ein_drop(in, pad);
        ein_ensure(in, 64);
        if (ein_avail(in) < 32u) goto leave;
        const uint32_t w = (uint32_t)in.bb;
        if ((w & 0xffffu) != ((w >> 16) ^ 0xffffu)) { rc = INF_DATA; goto done; }
        ein_drop(in, 32);
        uint32_t len = w & 0xffffu;
        for (; len; --len) {
          if (op == isize) goto leave;
          if ((++it & (TOK_K - 1u)) == 0u) ein_epoch(in);
          if (ein_short(in, 8)) { ++len; continue; }  // stall: retry this byte next epoch
          ein_refill(in);
          if (ein_avail(in) < 8u) goto leave;
          sink.literal(op++, (uint32_t)in.bb & 0xffu);
          ein_drop(in, 8);
        }
        continue;
      } else if (type == 1u) {
        // fixed Huffman code: lengths 8/9/7/8 for lit/len, 5 for distances
        uint32_t* l32 = (uint32_t*)(lens + TOK_LENS_LL);
        for (int s = 0; s < 288; s += 4) {
          const uint32_t v = s < 144 ? 8u : s < 256 ? 9u : s < 280 ? 7u : 8u;
          l32[s / 4] = v * 0x01010101u;
        }
        uint32_t* d32 = (uint32_t*)(lens + TOK_LENS_D);
        for (int s = 0; s < 32; s += 4) d32[s / 4] = 0x05050505u;
        Huff t;
        tok_build(lens + TOK_LENS_LL, 288, syms_ll, t, 1);
        huffp_make(t, hl);
        tok_build(lens + TOK_LENS_D, 32, syms_d, t, 2);
        huffp_make(t, hd);
      } else if (type == 2u) {
        ein_ensure(in, 64);
        if (ein_avail(in) < 14u) goto leave;
        const uint32_t nlen = ((uint32_t)in.bb & 31u) + 257u;
        const uint32_t ndist = ((uint32_t)(in.bb >> 5) & 31u) + 1u;
        const uint32_t ncode = ((uint32_t)(in.bb >> 10) & 15u) + 4u;
        ein_drop(in, 14);
        if (nlen > 286u || ndist > 30u) { rc = INF_DATA; goto done; }
        // 19 code-length code lengths (3 bits each, RFC 1951 order), at lens[0..19)
        const uint64_t ord_lo = 0x022caa324e804a30ULL, ord_hi = 0x00000003c2e1346cULL;
        {
          uint4* l4 = (uint4*)lens;
          l4[0] = make_uint4(0, 0, 0, 0);
          l4[1] = make_uint4(0, 0, 0, 0);
        }
        ein_ensure(in, 64);  // 19 * 3 = 57 bits at most
        for (uint32_t i = 0; i < ncode; ++i) {
          ein_refill(in);
          if (ein_avail(in) < 3u) goto leave;
          const uint32_t o = (uint32_t)((i < 12u ? ord_lo >> (5u * i) : ord_hi >> (5u * (i - 12u))) & 31u);
          lens[o] = (uint8_t)(in.bb & 7u);
          ein_drop(in, 3);
        }
        Huff hc;
        {
          Huff t;  // the build writes through a pointer; the decoder keeps its copy in registers
          if (!tok_build(lens, 19, syms_ll, t, 0)) { rc = INF_DATA; goto done; }
          hc = t;
        }
#ifdef HBAM_PROF
        TOK_PT(3);  // header bits + the code-length table
#endif
        // lit/len lengths -> lens[32 ..], distance lengths -> lens[320 ..].  The scratch is zeroed
        // first (20 quads), so a run of zero lengths (codes 17 / 18, up to 138 each) only advances
        // `have`; the loop is wave-uniform with the symbol loop's epoch clock (a per-lane clock put
        // an epoch, whose vmcnt(0) also waits for the last length's store, in nearly every
        // iteration of the divergent loop).
        const uint32_t total = nlen + ndist;
        {
          uint4* l4 = (uint4*)(lens + TOK_LENS_LL);
#pragma unroll
          for (int q = 0; q < (int)((TOK_LENS_END - TOK_LENS_LL) / 16u); ++q) l4[q] = make_uint4(0, 0, 0, 0);
        }
        uint32_t have = 0;
        uint32_t prev = 0;
        uint32_t hx = 0;  // 0 go on, 2 leave (zlib stops), 3 data error
        for (;;) {
          if ((__builtin_amdgcn_readfirstlane(++it) & (TOK_K - 1u)) == 0u) ein_epoch(in);
          const bool act = hx == 0u && have < total;
          if (__builtin_amdgcn_ballot_w64(act) == 0u) break;
          if (act && !ein_short(in, 14)) {
            ein_refill(in);
            uint32_t L = 1, sym = 0;
            if (hc.empty) {
              hx = ein_avail(in) < 1u ? 2u : 0u;
            } else {
              int32_t idx;
              huff_lookup(hc, ein_rev15(in), L, idx);  // CODES sets are complete
              if (L > ein_avail(in)) hx = 2u;
              else sym = syms_ll[idx];
            }
            if (hx == 0u) {
              if (sym < 16u) {
                ein_drop(in, L);
                lens[have < nlen ? TOK_LENS_LL + have : TOK_LENS_D + (have - nlen)] = (uint8_t)sym;
                ++have;
                prev = sym;
              } else {
                const uint32_t xb = sym == 16u ? 2u : sym == 17u ? 3u : 7u;
                if (L + xb > ein_avail(in)) {
                  hx = 2u;
                } else {
                  ein_drop(in, L);
                  if (sym == 16u && have == 0u) {
                    hx = 3u;
                  } else {
                    const uint32_t rep = sym == 16u ? 3u + ein_peek(in, 2) : sym == 17u ? 3u + ein_peek(in, 3)
                                                                                        : 11u + ein_peek(in, 7);
                    ein_drop(in, xb);
                    if (have + rep > total) {
                      hx = 3u;
                    } else {
                      if (sym == 16u)  // a repeat of the previous length (3-6); zeros are already there
                        for (uint32_t k = 0; k < rep; ++k)
                          lens[have + k < nlen ? TOK_LENS_LL + have + k : TOK_LENS_D + (have + k - nlen)] = (uint8_t)prev;
                      else
                        prev = 0;
                      have += rep;
                    }
                  }
                }
              }
            }
          }
        }
        if (hx == 2u) goto leave;
        if (hx == 3u) { rc = INF_DATA; goto done; }
#ifdef HBAM_PROF
        TOK_PT(4);  // the code lengths
#endif
        if (lens[TOK_LENS_LL + 256] == 0) { rc = INF_DATA; goto done; }
        {
          Huff t;
          if (!tok_build(lens + TOK_LENS_LL, (int)nlen, syms_ll, t, 1)) { rc = INF_DATA; goto done; }
          huffp_make(t, hl);
          if (!tok_build(lens + TOK_LENS_D, (int)ndist, syms_d, t, 2)) { rc = INF_DATA; goto done; }
          huffp_make(t, hd);
        }
#ifdef HBAM_PROF
        TOK_PT(5);  // the lit/len and distance tables
#endif
      } else {
        rc = INF_DATA;  // invalid block type
        goto done;
      }
    }
    // Drain the table copies (scratch) before the symbol loop: otherwise the loop carries
    // `s_waitcnt vmcnt(n)` on the distance tables into every iteration, which also waits for
    // the iteration's own output stores.
    __builtin_amdgcn_s_waitcnt(0);
    // ---- symbols of a Huffman-coded block
    // One structured loop (no continue / goto inside): every path of an iteration joins at
    // the loop's end with an exit code, so the decoder state needs no per-path copies.
    TOK_PT(6);  // header + tables
    {
      uint32_t ex = 0;  // 0 next symbol, 1 end of block, 2 leave (zlib stops), 3 data error
      TPend pd;
      pd.clear();
      // A wave-uniform loop (the exit is a ballot): a lane whose block has ended idles in it, as
      // it idled at the exit of a divergent loop, without the per-iteration exec-mask bookkeeping
      // of one.  The careful symbol (a lane's last 64 stream bits) runs behind a wave-uniform test.
      // With the predicated match mark and the branch-free bases: Huffman 31.1 -> 30.65 ms at
      // 5 GB, same output (profiles/r05/ab/huffman_uniform_loop_5g.txt).
      for (;;) {
        TOK_PC(0);
#ifdef HBAM_PROF
        TOK_PT(2);
#endif
        if ((__builtin_amdgcn_readfirstlane(++it) & (TOK_K - 1u)) == 0u) ein_epoch(in);
#ifdef HBAM_PROF
        TOK_PT(0);  // the epoch: merge (waits for the quad in flight) + the next request
#endif
        const bool run = ex == 0u && !ein_short(in, TOK_FAST_BITS);
        const bool fast = in.total - in.consumed >= TOK_FAST_BITS;
        if (run && fast) ex = tok_fast_spec(in, hl, hd, syms_ll, syms_d, sink, op, isize, pd);
        if (__builtin_amdgcn_ballot_w64(run && !fast) != 0u) {
          if (run && !fast) {
            pd.flush(sink);
            ex = tok_careful(in, hl, hd, syms_ll, syms_d, sink, op, isize);
          }
        }
#ifdef HBAM_PROF
        TOK_PT(1);
#endif
        if (__builtin_amdgcn_ballot_w64(ex == 0u) == 0u) break;
      }
      pd.flush(sink);  // the last fast iteration's packet and mark
      if (ex == 2u) goto leave;
      if (ex == 3u) {
        rc = INF_DATA;
        goto done;
      }
    }
  }
leave:
  rc = (op == isize) ? INF_OK : INF_SHORT;
done:
  sink.finish();
  *produced = op;
#ifdef HBAM_PROF
  // decoder state at exit (tools/diag_inflate_build.py)
  pc[1] = in.consumed;
  pc[2] = in.bc | in.nv << 8 | in.rd << 16;
  pc[3] = it;
#endif
  return rc;
}

}  // namespace hbam
