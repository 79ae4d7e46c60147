// hbam_sort.hip — device side of the coordinate Sort plugin path.
//
// Replaces the MapReduce shuffle sort of Sort.java:84-188 (SortRecordReader keys records with
// BAMRecordReader.getKey, Sort.java:279-295; Hadoop sorts LongWritable keys as SIGNED i64;
// SortReducer is the identity, Sort.java:191-205).  The reference's tie order is unspecified
// (unstable spill QuickSort + merge); this path defines it as input order, i.e. (key, file,
// voffset), by sorting stably.
//
// Layout: keys are sorted as u64 with the sign bit flipped (signed order == unsigned order of
// key ^ 1<<63), carrying a u32 record index.  LSD radix, 8-bit digits, up to 8 passes; a pass
// whose digit is the same for every key is skipped (one fused 8-digit histogram decides, so a
// coordinate key — refID in the high word, small — usually needs 4-5 passes).
// Per pass: k_rs_count (per-tile digit counts, digit-major) -> exclusive scan (shared with the
// decode path) -> k_rs_scatter (stable in-tile ranking: 64-lane ballot match per 8-bit digit,
// cross-wave prefix through LDS, one round of 256 keys at a time so the rank follows index
// order).  All HBM traffic is streamed: 12 B read twice + 12 B written per key per pass.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hbam {

constexpr uint32_t RS_WG = 256;
constexpr uint32_t RS_IPT = 16;
constexpr uint32_t RS_TILE = RS_WG * RS_IPT;
constexpr uint64_t RS_SIGN = 0x8000000000000000ull;

__global__ __launch_bounds__(RS_WG) void k_rs_init(const int64_t* __restrict__ keys, uint64_t n,
                                                   uint64_t* __restrict__ ukeys,
                                                   uint32_t* __restrict__ idx,
                                                   uint32_t* __restrict__ hist8) {
  __shared__ uint32_t h[8][256];
  for (uint32_t k = threadIdx.x; k < 8 * 256; k += RS_WG) (&h[0][0])[k] = 0;
  __syncthreads();
  const uint64_t stride = (uint64_t)gridDim.x * RS_WG;
  for (uint64_t i = (uint64_t)blockIdx.x * RS_WG + threadIdx.x; i < n; i += stride) {
    const uint64_t u = (uint64_t)keys[i] ^ RS_SIGN;
    ukeys[i] = u;
    idx[i] = (uint32_t)i;
#pragma unroll
    for (uint32_t d = 0; d < 8; ++d) atomicAdd(&h[d][(u >> (8 * d)) & 255u], 1u);
  }
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < 8 * 256; k += RS_WG) {
    const uint32_t v = (&h[0][0])[k];
    if (v) atomicAdd(hist8 + k, v);
  }
}

__global__ __launch_bounds__(RS_WG) void k_rs_count(const uint64_t* __restrict__ kin, uint64_t n,
                                                    uint32_t shift, uint32_t ntiles,
                                                    uint32_t* __restrict__ counts) {
  __shared__ uint32_t h[256];
  h[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t base = (uint64_t)blockIdx.x * RS_TILE;
#pragma unroll 4
  for (uint32_t r = 0; r < RS_IPT; ++r) {
    const uint64_t i = base + r * RS_WG + threadIdx.x;
    if (i < n) atomicAdd(&h[(kin[i] >> shift) & 255u], 1u);
  }
  __syncthreads();
  counts[(uint64_t)threadIdx.x * ntiles + blockIdx.x] = h[threadIdx.x];
}

__global__ __launch_bounds__(RS_WG) void k_rs_scatter(const uint64_t* __restrict__ kin,
                                                      const uint32_t* __restrict__ vin, uint64_t n,
                                                      uint32_t shift, uint32_t ntiles,
                                                      const uint64_t* __restrict__ off,
                                                      uint64_t* __restrict__ kout,
                                                      uint32_t* __restrict__ vout) {
  __shared__ uint64_t gb[256];
  __shared__ uint32_t run[256];
  __shared__ uint32_t wc[RS_WG / 64][256];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, w = tid >> 6;
  gb[tid] = off[(uint64_t)tid * ntiles + blockIdx.x];
  run[tid] = 0;
#pragma unroll
  for (uint32_t q = 0; q < RS_WG / 64; ++q) wc[q][tid] = 0;
  __syncthreads();
  const uint64_t base = (uint64_t)blockIdx.x * RS_TILE;
  const uint64_t lt = (1ull << lane) - 1ull;
  for (uint32_t r = 0; r < RS_IPT; ++r) {
    const uint64_t i = base + r * RS_WG + tid;
    const bool valid = i < n;
    const uint64_t k = valid ? kin[i] : 0;
    const uint32_t v = valid ? vin[i] : 0;
    const uint32_t dig = (uint32_t)(k >> shift) & 255u;
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (uint32_t b = 0; b < 8; ++b) {
      const bool bit = (dig >> b) & 1u;
      const uint64_t m = __ballot(bit);
      peers &= bit ? m : ~m;
    }
    const uint32_t rank = (uint32_t)__popcll(peers & lt);
    if (valid && (peers & lt) == 0) wc[w][dig] = (uint32_t)__popcll(peers);
    __syncthreads();
    if (valid) {
      uint32_t pos = run[dig] + rank;
      for (uint32_t q = 0; q < w; ++q) pos += wc[q][dig];
      const uint64_t dst = gb[dig] + pos;
      kout[dst] = k;
      vout[dst] = v;
    }
    __syncthreads();
    uint32_t s = 0;
#pragma unroll
    for (uint32_t q = 0; q < RS_WG / 64; ++q) {
      s += wc[q][tid];
      wc[q][tid] = 0;
    }
    run[tid] += s;
    __syncthreads();
  }
}

__global__ __launch_bounds__(RS_WG) void k_rs_finish(const uint64_t* __restrict__ ukeys, uint64_t n,
                                                     int64_t* __restrict__ keys_out) {
  const uint64_t i = (uint64_t)blockIdx.x * RS_WG + threadIdx.x;
  if (i < n) keys_out[i] = (int64_t)(ukeys[i] ^ RS_SIGN);
}

template <typename T>
__global__ __launch_bounds__(RS_WG) void k_permute(const T* __restrict__ src,
                                                   const uint32_t* __restrict__ perm, uint64_t n,
                                                   T* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * RS_WG + threadIdx.x;
  if (i < n) out[i] = src[perm[i]];
}

// record payload lengths (SAMRecordWritable wire form: block_size field + record) in perm order
__global__ __launch_bounds__(RS_WG) void k_perm_lens(const int32_t* __restrict__ block_size,
                                                     const uint32_t* __restrict__ perm, uint64_t n,
                                                     uint32_t* __restrict__ lens) {
  const uint64_t i = (uint64_t)blockIdx.x * RS_WG + threadIdx.x;
  if (i < n) lens[i] = 4u + (uint32_t)block_size[perm ? perm[i] : i];
}

// The record gather (SAMRecordWritable payloads in permutation order), a wave per tile of 64
// consecutive output records (k_decode_pools' unit
// scheme): each lane reads its record's source offset and length once, every record is cut into
// 16-byte units numbered by a wave scan, and consecutive lanes take consecutive units (a unit's
// record found by popcount, below), so a wave instruction moves ~1 KiB of the output
// stream and the three dependent index loads are paid once per 64 records instead of once per
// record.  A record's last unit may be shorter: written in 8/4/2/1-byte pieces, so a neighbour's
// bytes are never written.  Source over-reads (up to 15 bytes past a record) stay inside ubuf +
// its slack.
__global__ __launch_bounds__(256) void k_gather_records_tile(const uint8_t* __restrict__ ubuf,
                                                             const uint64_t* __restrict__ rec_off,
                                                             const uint32_t* __restrict__ perm, uint64_t n,
                                                             const uint64_t* __restrict__ out_off,
                                                             uint8_t* __restrict__ out) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t ntiles = (n + 63) / 64;
  const uint64_t wstride = (uint64_t)gridDim.x * (blockDim.x / 64);
  // The pools kernel's unit mapping (hbam_kernels.hip, k_decode_pools): DPP scans, each record's
  // (source, destination, bytes, first unit) once in LDS at its rank, a unit's record by popcount;
  // two 64-unit windows per step with both loads (random sources: the permuted records) and their
  // wait in one asm statement.  Against the shuffle-search form: sort + pack 14.2 -> 13.4 ms at
  // 5 GB, the same order and payloads (profiles/r05/ab/sort_gather_5g_*.json).
  __shared__ uint4 s_rec[4][64];
  __shared__ uint32_t s_first[4][64];
  uint4* const recs = s_rec[threadIdx.x >> 6];
  uint32_t* const firsts = s_first[threadIdx.x >> 6];
  const uint64_t le = lane == 63u ? ~0ull : ((2ull << lane) - 1ull);
  for (uint64_t t = (uint64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); t < ntiles; t += wstride) {
    const uint64_t i = t * 64 + lane;
    uint64_t src = 0, dst = 0;
    uint32_t len = 0;
    if (i < n) {
      src = rec_off[perm ? perm[i] : i];
      dst = out_off[i];
      len = (uint32_t)(out_off[i + 1] - dst);
    }
    const uint32_t units = (len + 15u) >> 4;
    const uint32_t incl = wave_scan_dpp(units), excl = incl - units, total = wave_last(incl);
    if (total == 0u) continue;
    const bool has = units != 0u;
    const uint64_t mh = __ballot(has);
    const uint32_t first = (uint32_t)__builtin_ctzll(mh);
    const uint64_t db = readlane64(dst, first);  // (zero-extends the low half: dst passes 2^31)
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");  // the previous tile's reads of the table precede these writes
    if (has) {
      const uint32_t rk = lane_rank(mh);
      recs[rk] = make_uint4((uint32_t)src, (uint32_t)(src >> 32), (uint32_t)(dst - db), len);
      firsts[rk] = excl;
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    uint8_t* const obase = out + db;
    for (uint32_t q0 = 0; q0 < total; q0 += 128) {
      u32x4_t raw[2];
      const uint8_t* sp[2];
      uint8_t* dp[2];
      uint32_t nn[2];
#pragma unroll
      for (uint32_t w = 0; w < 2; ++w) {
        nn[w] = 0;
        dp[w] = obase;
        sp[w] = ubuf;  // valid dummy address
        const uint32_t qw = q0 + 64u * w;
        if (qw >= total) continue;  // wave-uniform
        const uint32_t q = qw + lane;
        const uint32_t pos = excl - qw;
        const bool inwin = has && excl >= qw && pos < 64u;
        const uint32_t blo = (inwin && pos < 32u) ? 1u << pos : 0u;
        const uint32_t bhi = (inwin && pos >= 32u) ? 1u << (pos - 32u) : 0u;
        const uint64_t M = (uint64_t)wave_last(wave_scan_dpp(bhi)) << 32 | wave_last(wave_scan_dpp(blo));
        const uint32_t c0 = (uint32_t)__popcll(__ballot(has && excl < qw));
        if (q < total) {
          const uint32_t rk = c0 + (uint32_t)__popcll(M & le) - 1u;
          const uint4 rr = recs[rk];
          const uint32_t k = q - firsts[rk];
          nn[w] = rr.w - 16u * k;
          dp[w] = obase + rr.z + 16u * k;
          sp[w] = ubuf + ((uint64_t)rr.x | (uint64_t)rr.y << 32) + 16u * k;
        }
      }
      asm volatile("global_load_dwordx4 %0, %2, off\n\tglobal_load_dwordx4 %1, %3, off\n\ts_waitcnt vmcnt(0)"
                   : "=&v"(raw[0]), "=&v"(raw[1]) : "v"(sp[0]), "v"(sp[1]) : "memory");
#pragma unroll
      for (uint32_t w = 0; w < 2; ++w) {
        if (q0 + 64u * w >= total) break;  // wave-uniform
        const u32x4_a1 v = u32x4_a1{raw[w][0], raw[w][1], raw[w][2], raw[w][3]};
        HBAM_G uint8_t* const gd = (HBAM_G uint8_t*)dp[w];
        if (nn[w] >= 16u) *(HBAM_G u32x4_a1*)gd = v;
        else if (nn[w] != 0u) st_part_g(gd, nn[w], v);
      }
    }
  }
}

// TotalOrderPartitioner bounds: for split point j, the first index whose (signed) key is
// greater (partition j holds keys <= sp[j]); sorted keys, one thread per split point
__global__ __launch_bounds__(RS_WG) void k_sort_bounds(const int64_t* __restrict__ keys, uint64_t n,
                                                       const int64_t* __restrict__ sp, uint32_t m,
                                                       const uint64_t* __restrict__ offsets,
                                                       uint64_t* __restrict__ rec_b,
                                                       uint64_t* __restrict__ byte_b) {
  const uint32_t j = blockIdx.x * RS_WG + threadIdx.x;
  if (j >= m) return;
  const int64_t v = sp[j];
  uint64_t lo = 0, hi = n;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (keys[mid] <= v) lo = mid + 1;
    else hi = mid;
  }
  rec_b[j] = lo;
  byte_b[j] = offsets[lo];
}

// InputSampler stand-in of the exchange (Sort.java:154-157): regular
// samples of a rank's sorted keys, out[0] = k = min(n, s), out[1 + j] = keys[j * n / k]
__global__ __launch_bounds__(RS_WG) void k_sample_keys(const int64_t* __restrict__ keys, uint64_t n,
                                                       uint32_t s, int64_t* __restrict__ out) {
  const uint64_t k = n < (uint64_t)s ? n : (uint64_t)s;
  const uint32_t j = blockIdx.x * RS_WG + threadIdx.x;
  if (j == 0) out[0] = (int64_t)k;
  if (j < s) out[1 + j] = j < k ? keys[(uint64_t)j * n / k] : 0;
}

// SplittingBAMIndexer (SplittingBAMIndexer.java:146-248): the voffset before every
// granularity-th record (records counted from 1) of a whole-file decode
__global__ __launch_bounds__(RS_WG) void k_index_pick(const uint64_t* __restrict__ voffset, uint64_t n,
                                                      uint32_t g, uint64_t* __restrict__ out) {
  const uint64_t j = (uint64_t)blockIdx.x * RS_WG + threadIdx.x;  // output entry j: record (j+1)*g-1
  const uint64_t r = (j + 1) * (uint64_t)g - 1;
  if (r < n) out[j] = voffset[r];
}

// BGZFBlockIndexer.index (util/BGZFBlockIndexer.java:109-122): entry j = the indexer's int
// `pos` after block (j+1)*g, i.e. the next block's offset (or the file length after the last
// block), as the low 48 bits of the sign-extended Java int (wraps past 2 GiB, :88,115-116).
__global__ __launch_bounds__(RS_WG) void k_bgzfi_pick(const BlockRec* __restrict__ blk, uint64_t nb,
                                                      uint64_t file_len, uint32_t g,
                                                      uint64_t k, uint64_t* __restrict__ out) {
  const uint64_t j = (uint64_t)blockIdx.x * RS_WG + threadIdx.x;
  if (j >= k) return;
  const uint64_t b = (j + 1) * (uint64_t)g;
  const uint64_t p = b < nb ? blk[b].coff : file_len;
  out[j] = (uint64_t)(int64_t)(int32_t)(uint32_t)p & 0xffffffffffffull;
}

// Multi-input Sort: SortRecordReader.nextKeyValue (Sort.java:279-295) applies
// Utils.correctSAMRecordForMerging (cli/Utils.java:286-313) to every record when the inputs'
// dictionaries differ: refID -> the merged index, next refID too for a paired read (0x1), in
// the record's bytes (SAMRecordWritable.write encodes them) and the columns, and the key
// recomputed by BAMRecordReader.getKey when refID changed.  getKey's hash (unmapped records) is
// over the variable block, which a refID change leaves as it is, so only coordinate keys move.
// htsjdk's SAMRecord.setReferenceIndex / setMateReferenceIndex resolve the new index against
// the record's OWN (input) header and throw IllegalArgumentException when it is beyond that
// dictionary: the first such record -> *first_bad.
__global__ __launch_bounds__(RS_WG) void k_merge_remap(uint8_t* __restrict__ ubuf,
                                                       const uint64_t* __restrict__ rec_off, uint64_t n,
                                                       int32_t* __restrict__ ref_col,
                                                       int32_t* __restrict__ nref_col,
                                                       int64_t* __restrict__ key_col,
                                                       const uint16_t* __restrict__ flag_col,
                                                       const int32_t* __restrict__ pos_col,
                                                       const int32_t* __restrict__ map, int32_t n_in,
                                                       unsigned long long* __restrict__ first_bad) {
  const uint64_t i = (uint64_t)blockIdx.x * RS_WG + threadIdx.x;
  if (i >= n) return;
  auto remap = [&](int32_t x) { return x == -1 ? -1 : (x >= 0 && x < n_in) ? map[x] : n_in; };
  const int32_t r = ref_col[i], m = nref_col[i];
  const uint16_t f = flag_col[i];
  const int32_t nr = remap(r);
  const int32_t nm = (f & 1u) ? remap(m) : m;
  if (nr >= n_in || ((f & 1u) && nm >= n_in)) {
    atomicMin(first_bad, (unsigned long long)i);
    return;
  }
  uint8_t* p = ubuf + rec_off[i];
  if (nr != r) {
    for (int k = 0; k < 4; ++k) p[4 + k] = (uint8_t)((uint32_t)nr >> (8 * k));
    ref_col[i] = nr;
    const int32_t pos = pos_col[i];
    if (!(f & 4u) && nr >= 0 && (int32_t)((uint32_t)pos + 1u) >= 0)
      key_col[i] = (int64_t)((uint64_t)(int64_t)nr << 32 | (uint64_t)(int64_t)pos);
  }
  if (nm != m) {
    for (int k = 0; k < 4; ++k) p[24 + k] = (uint8_t)((uint32_t)nm >> (8 * k));
    nref_col[i] = nm;
  }
}

}  // namespace hbam
