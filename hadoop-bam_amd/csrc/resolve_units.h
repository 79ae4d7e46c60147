// resolve_units.h — LZ77 resolution by 16-byte units (k_resolve_units), gfx950.
//
// Input / output / error contract: resolve_dev.h.  One wave per BGZF block walks the block in
// RS_S-byte stretches staged in LDS with an RS_W-byte window behind.  The round-4 kernel (k_resolve,
// commit 88cff91) copied a whole match per lane, so a wave-step ran the union of every lane's copy
// loop (period < 8, 32-byte groups, 8-byte chunks) and every partial write was a misaligned
// ds_write_b64/b32/b16/b8 behind its own branch: the LDS pipe spent ~27 % of its cycles in
// misaligned-access replays and the exec-mask bookkeeping was as many scalar instructions as there
// were vector ones (round-4 SQ counters).
//
// Here every match is cut, when its descriptor is read, into units of at most 16 bytes whose
// source never overlaps their own destination:
//   * dist >= len, or dist >= 16: units of 16 bytes at distance dist;
//   * dist < 8 (< len): a head unit of min(16, len) bytes built from the dist-byte period (v_perm
//     over the first 8 source bytes), then units at distance dist * ceil(16 / dist) >= 16;
//   * 8 <= dist < 16 (< len): a head unit of dist bytes, then units at distance 2 * dist.
// A unit is one straight-line copy: a 16-byte read from a dword-aligned b128 + b32 pair (or one
// global load for a source older than the window) and five aligned ds_mskor_b32 writes
// (D = (D & ~mask) | data), so neighbouring units' bytes in one dword never clobber each other and
// no access is misaligned.  Units of "pre" matches (source final before the stretch) are all
// independent; the others run as k_resolve's dataflow rounds over units instead of matches
// (tools/unit_sim.py: the same rounds, 30 units per stretch against 28 matches).
//
// Included by hbam_kernels.hip inside namespace hbam, after rs_write_back.
#pragma once

// units per stretch: matches are >= 3 bytes and disjoint, and a unit covers >= 3 bytes of its
// match except the last: 342 matches starting in a stretch, plus the 17 extra units of a final
// 258-byte match, at most
constexpr uint32_t RU_CAP = 360;
// RU_CAP and the 11-bit destination field of a unit record (rel < RS_S + 258 <= 2047) are sized for
// 1 KiB stretches: a 2 KiB stretch would overrun both silently
static_assert(RS_S == 1024, "k_resolve_units: unit capacity and record packing assume 1 KiB stretches");

// unit record: bits 0-10 destination - s0 (< RS_S + 258), 11-14 bytes - 1, 15-29 distance - 1,
// bit 30: periodic head unit (distance < 8 < bytes)
__device__ __forceinline__ uint32_t ru_pack(uint32_t rel, uint32_t n, uint32_t dist, bool per) {
  return rel | (n - 1u) << 11 | (dist - 1u) << 15 | (per ? 1u << 30 : 0u);
}

// 16 bytes at LDS byte index x, from a dword-aligned b128 + b32 (full rate) and v_alignbit
__device__ __forceinline__ uint4 ru_rd16(const uint8_t* buf, uint32_t x) {
  uint32_t a = x & ~3u;
  const uint32_t sh = (x & 3u) * 8u;
  // hide the 4-byte alignment from the compiler, which would otherwise split the read into a
  // misaligned ds_read_b64 + ds_read2_b32: one ds_read_b128 at dword alignment runs at full rate
  asm("" : "+v"(a));
  // an ext_vector load carries align 16 in the IR (uint4 is a struct of four u32: align 4, which
  // the backend split into ds_read_b64 + ds_read2_b32 pairs; A/B at 5 GB, with the scalar-mask
  // rounds below: 15.52 -> 15.34 ms, profiles/r05/ab/resolve_sround_b128_5g.txt)
  const u32x4_t qv = *(const u32x4_t*)(buf + a);
  const uint4 q = make_uint4(qv[0], qv[1], qv[2], qv[3]);
  const uint32_t q4 = *(const uint32_t*)(buf + a + 16u);
  return make_uint4(__builtin_amdgcn_alignbit(q.y, q.x, sh), __builtin_amdgcn_alignbit(q.z, q.y, sh),
                    __builtin_amdgcn_alignbit(q.w, q.z, sh), __builtin_amdgcn_alignbit(q4, q.w, sh));
}

__device__ __forceinline__ uint32_t ru_lowbytes(uint32_t k) {  // mask of the low k (0..4) bytes
  return k >= 4u ? ~0u : (1u << (8u * k)) - 1u;
}

// bytes [0, n) of v (1 <= n <= 16) to LDS byte index x: five dword-aligned ds_mskor_b32
__device__ __forceinline__ void ru_put(uint8_t* buf, uint32_t x, uint32_t n, const uint4 v) {
  const uint32_t o = x & 3u, e = o + n, rs = 32u - 8u * o;
  const uint32_t addr = (uint32_t)(uintptr_t)(buf + (x & ~3u));
  const uint32_t d0 = v.x << (8u * o);
  const uint32_t d1 = (uint32_t)((((uint64_t)v.y << 32) | v.x) >> rs);
  const uint32_t d2 = (uint32_t)((((uint64_t)v.z << 32) | v.y) >> rs);
  const uint32_t d3 = (uint32_t)((((uint64_t)v.w << 32) | v.z) >> rs);
  const uint32_t d4 = (uint32_t)((uint64_t)v.w >> rs);
  const uint32_t m0 = ru_lowbytes(e < 4u ? e : 4u) & ~ru_lowbytes(o);
  const uint32_t m1 = ru_lowbytes(e > 4u ? e - 4u : 0u);
  const uint32_t m2 = ru_lowbytes(e > 8u ? e - 8u : 0u);
  const uint32_t m3 = ru_lowbytes(e > 12u ? e - 12u : 0u);
  const uint32_t m4 = ru_lowbytes(e > 16u ? e - 16u : 0u);
  // dwords 0-1 always (a unit covers >= 1 byte, and the no-op mask is harmless); 2-4 only for
  // the lanes whose bytes reach them (an inactive lane costs the LDS nothing)
  asm volatile(
      "ds_mskor_b32 %0, %1, %2\n\t"
      "ds_mskor_b32 %0, %3, %4 offset:4"
      :
      : "v"(addr), "v"(m0), "v"(d0 & m0), "v"(m1), "v"(d1 & m1)
      : "memory");
  if (e > 8u) asm volatile("ds_mskor_b32 %0, %1, %2 offset:8" : : "v"(addr), "v"(m2), "v"(d2 & m2) : "memory");
  if (e > 12u) asm volatile("ds_mskor_b32 %0, %1, %2 offset:12" : : "v"(addr), "v"(m3), "v"(d3 & m3) : "memory");
  if (e > 16u) asm volatile("ds_mskor_b32 %0, %1, %2 offset:16" : : "v"(addr), "v"(m4), "v"(d4 & m4) : "memory");
}

// bytes j < 16 of the period-d (1..7) sequence whose first d bytes are the low bytes of v
__device__ __forceinline__ uint4 ru_periodic(uint4 v, uint32_t d, const uint4* __restrict__ sel) {
  const uint4 s = sel[d];
  return make_uint4(__builtin_amdgcn_perm(v.y, v.x, s.x), __builtin_amdgcn_perm(v.y, v.x, s.y),
                    __builtin_amdgcn_perm(v.y, v.x, s.z), __builtin_amdgcn_perm(v.y, v.x, s.w));
}

// the same with all five writes issued (a dword the unit does not reach gets mask 0: D unchanged),
// so the caller's exec mask needs no per-dword branches
__device__ __forceinline__ void ru_put5(uint8_t* buf, uint32_t x, uint32_t n, const uint4 v) {
  const uint32_t o = x & 3u, e = o + n, rs = 32u - 8u * o;
  const uint32_t addr = (uint32_t)(uintptr_t)(buf + (x & ~3u));
  const uint32_t d0 = v.x << (8u * o);
  const uint32_t d1 = (uint32_t)((((uint64_t)v.y << 32) | v.x) >> rs);
  const uint32_t d2 = (uint32_t)((((uint64_t)v.z << 32) | v.y) >> rs);
  const uint32_t d3 = (uint32_t)((((uint64_t)v.w << 32) | v.z) >> rs);
  const uint32_t d4 = (uint32_t)((uint64_t)v.w >> rs);
  const uint32_t m0 = ru_lowbytes(e < 4u ? e : 4u) & ~ru_lowbytes(o);
  const uint32_t m1 = ru_lowbytes(e > 4u ? e - 4u : 0u);
  const uint32_t m2 = ru_lowbytes(e > 8u ? e - 8u : 0u);
  const uint32_t m3 = ru_lowbytes(e > 12u ? e - 12u : 0u);
  const uint32_t m4 = ru_lowbytes(e > 16u ? e - 16u : 0u);
  asm volatile(
      "ds_mskor_b32 %0, %1, %2\n\t"
      "ds_mskor_b32 %0, %3, %4 offset:4\n\t"
      "ds_mskor_b32 %0, %5, %6 offset:8\n\t"
      "ds_mskor_b32 %0, %7, %8 offset:12\n\t"
      "ds_mskor_b32 %0, %9, %10 offset:16"
      :
      : "v"(addr), "v"(m0), "v"(d0 & m0), "v"(m1), "v"(d1 & m1), "v"(m2), "v"(d2 & m2), "v"(m3),
        "v"(d3 & m3), "v"(m4), "v"(d4 & m4)
      : "memory");
}

// one unit: its 16-byte source (LDS, final) -> its destination
template <bool ALL5 = false>
__device__ __forceinline__ void ru_copy(uint8_t* __restrict__ buf, uint32_t di, uint32_t n, uint32_t dist,
                                        bool per, const uint4* __restrict__ sel) {
  uint4 v = ru_rd16(buf, di - dist);
  if (per) v = ru_periodic(v, dist, sel);
  if (ALL5) ru_put5(buf, di, n, v);
  else ru_put(buf, di, n, v);
}

constexpr uint32_t RU_WAVES = 8;  // waves per SIMD (the LDS allows 8 at 4.9 KiB per block)

__global__ __launch_bounds__(64, RU_WAVES) void k_resolve_units(const BlockRec* __restrict__ blk,
                                                                     const uint64_t* __restrict__ uoff, uint32_t nblk,
                                                                     uint8_t* __restrict__ ubuf,
                                                                     const uint32_t* __restrict__ bitmap,
                                                                     const uint32_t* __restrict__ tails,
                                                                     int32_t* __restrict__ status) {
  __shared__ __attribute__((aligned(16))) uint8_t s_buf[RS_BUF];
  __shared__ uint32_t s_unit[RU_CAP];  // pre units from the front, ordered units from the back
  __shared__ uint16_t s_pos[RS_MAXM];
  __shared__ uint4 s_sel[8];  // row d: byte j = j mod d (v_perm selectors over 8 source bytes)
  __shared__ uint32_t s_pend[RS_PW];
  const uint32_t b = blockIdx.x;
  const uint32_t lane = threadIdx.x;
  if (b >= nblk) return;
#ifdef HBAM_PROF
  const uint64_t pr0 = PROF_RT(), pc0 = PROF_CLK();
  uint64_t p_desc = 0, p_bat = 0, n_bat = 0, n_m = 0, p_st = 0, p_pre = 0, p_wb = 0;
#endif
  if (status[b] != INF_OK) return;
  const uint32_t isize = blk[b].isize;
  if (isize == 0 || isize > 65536u) return;
  const uint32_t* bm = bitmap + (uint64_t)b * BITMAP_WORDS;
  const uint32_t nwords = (isize + 31u) >> 5;
  const uint32_t tail0 = tails[2 * (uint64_t)b];
  {
    uint32_t any = 0;
    for (uint32_t w = lane; w < nwords; w += 64) any |= bm[w];
    if (!__any(any != 0) && !(tail0 & 0x80000000u)) return;
  }
  if (lane < 32) {
    const uint32_t d = (lane >> 2) ? (lane >> 2) : 1u, q = lane & 3u;
    uint32_t s = 0;
    for (uint32_t j = 0; j < 4; ++j) s |= ((4u * q + j) % d) << (8 * j);
    ((uint32_t*)s_sel)[lane] = s;
  }
  const uint64_t base = uoff[b];
  const uint64_t abase = base & ~15ULL;
  const uint32_t a0 = (uint32_t)(base - abase);
  const uint64_t aend = base + isize;
  const uint32_t nstr = (a0 + isize + RS_S - 1) / RS_S;
  auto load_raw = [&](uint32_t k, uint4& r0, uint4& r1) {
    const uint64_t g = abase + (uint64_t)k * RS_S + 16u * lane;
    if (k < nstr) {
      r0 = *(const uint4*)(ubuf + g);
      if (RS_C == 2) r1 = *(const uint4*)(ubuf + g + 1024);
    }
  };
  uint4 ra0 = make_uint4(0, 0, 0, 0), ra1 = ra0, rb0 = ra0, rb1 = ra0;
  load_raw(0, ra0, ra1);
  load_raw(1, rb0, rb1);
  *(uint4*)(s_buf + RS_W + 16u * lane) = ra0;
  if (RS_C == 2) *(uint4*)(s_buf + RS_W + 1024 + 16u * lane) = ra1;
  *(uint4*)(s_buf + RS_W + RS_S + 16u * lane) = rb0;
  if (RS_C == 2) *(uint4*)(s_buf + RS_W + RS_S + 1024 + 16u * lane) = rb1;
  constexpr uint32_t WPS = RS_S / 32;
  uint32_t wcur = (lane < WPS && lane < nwords) ? bm[lane] : 0u;
  __syncthreads();
  asm volatile("" : "+v"(wcur));  // defined here for the compiler's wait tracking (see the drain below)
#ifdef HBAM_PROF
  p_st = PROF_CLK() - pc0;
#endif
  for (uint32_t k = 0; k < nstr; ++k) {
    const uint32_t s0 = k * RS_S;
#ifdef HBAM_PROF
    const uint64_t q0 = PROF_CLK();
#endif
    // this stretch's bitmap words: requested before the previous stretch's drain and in registers
    // since (a load issued here would make the compiler wait for every store of the last write-back)
    const uint32_t word = wcur;
    const uint32_t lbase = RS_W + a0 - s0;  // LDS index of block offset x: x + lbase
    // ---- match starts of the stretch -> s_pos (in order)
    const uint32_t cnt = __popc(word);
    const uint32_t incl = wave_scan_dpp(cnt);
    const uint32_t total = wave_last(incl);
    {
      uint32_t wpos = incl - cnt, bits = word;
      while (bits) {
        const uint32_t bit = __ffs(bits) - 1;
        bits &= bits - 1;
        s_pos[wpos++] = (uint16_t)(s0 + 32u * lane + bit);
      }
    }
    __syncthreads();
    // ---- descriptors -> units, split pre (all independent) / ordered (dataflow)
    uint32_t npre = 0, nord = 0;
    bool bad_desc = false;
    for (uint32_t j0 = 0; j0 < total; j0 += 64) {
      const uint32_t j = j0 + lane;
      uint32_t p = 0, len = 0, dist = 1, nu = 0, h = 0, D = 1;
      bool pre = false, per = false;
      if (j < total) {
        p = s_pos[j];
        const uint32_t dsc = lds_rd32u(s_buf, lbase + p);
        len = (dsc & 0xffu) + 3u;
        dist = ((dsc >> 8) & 0xffffu) + 1u;
        const uint32_t e = p - dist + (len < dist ? len : dist);
        bad_desc |= dist > p || p + len > isize || dist > 32768u;
        pre = dist >= len && e <= s0;
        if (dist >= len || dist >= 16u) {
          D = dist;
        } else if (dist < 8u) {
          h = len < 16u ? len : 16u;
          // dist * ceil(16 / dist) for dist 1..7 = 16 + {0,0,0,2,0,4,2,5}[dist] (no integer division)
          D = 16u + ((0xAA0400u >> (3u * dist)) & 7u);
          per = true;
        } else {
          h = dist;
          D = 2u * dist;
        }
        nu = (h ? 1u : 0u) + (len - h + 15u) / 16u;
      }
      const uint32_t up = pre ? nu : 0u, uo = pre ? 0u : nu;
      const uint32_t ipo = wave_scan_dpp(up | uo << 16);  // both counts in one scan (each < 2^16)
      const uint32_t ip = ipo & 0xffffu, io = ipo >> 16;
      if (up) {
        const uint32_t w = npre + ip - up;
        for (uint32_t u = 0; u < up; ++u)
          s_unit[w + u] = ru_pack(p - s0 + 16u * u, len - 16u * u < 16u ? len - 16u * u : 16u, dist, false);
      } else if (uo) {
        const uint32_t w = nord + io - uo;
        uint32_t u = 0;
        if (h) s_unit[RU_CAP - 1u - (w + u++)] = ru_pack(p - s0, h, dist, per);
        for (uint32_t q = p + h; u < uo; ++u, q += 16u)
          s_unit[RU_CAP - 1u - (w + u)] = ru_pack(q - s0, p + len - q < 16u ? p + len - q : 16u, D, false);
      }
      const uint32_t tpo = wave_last(ipo);
      npre += tpo & 0xffffu;
      nord += tpo >> 16;
    }
    if (__any(bad_desc)) {  // never copy from outside the block: report DataFormatException
      if (lane == 0) status[b] = INF_DATA;
      return;
    }
    __syncthreads();
#ifdef HBAM_PROF
    const uint64_t q1 = PROF_CLK();
    p_desc += q1 - q0;
    n_m += total;
#endif
    // ---- pre units: every source final (the LDS window, or ubuf written back at least one
    // iteration ago, which the drain makes visible).  The next stretch's bitmap words are
    // requested first, so they land with the drain.
    {
      const uint32_t wi = (k + 1) * WPS + lane;
      wcur = (lane < WPS && k + 1 < nstr && wi < nwords) ? bm[wi] : 0u;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("" : "+v"(wcur));  // the next stretch's words land with the drain
    // two units per lane per step, both sources requested before either is written: the far
    // (global) reads of a step are in flight together
    for (uint32_t i = lane; i < npre; i += 128) {
      const bool two = i + 64u < npre;
      const uint32_t r = s_unit[i], r2 = two ? s_unit[i + 64u] : 0u;
      const uint32_t q = s0 + (r & 2047u), dist = ((r >> 15) & 0x7fffu) + 1u;
      const uint32_t q2 = s0 + (r2 & 2047u), dist2 = ((r2 >> 15) & 0x7fffu) + 1u;
      const uint32_t src = q - dist, src2 = q2 - dist2;
      uint4 v, v2 = make_uint4(0, 0, 0, 0);
      if (src + RS_W + a0 >= s0) v = ru_rd16(s_buf, lbase + src);
      else v = *(const uint4*)(ubuf + base + src);
      if (two) {
        if (src2 + RS_W + a0 >= s0) v2 = ru_rd16(s_buf, lbase + src2);
        else v2 = *(const uint4*)(ubuf + base + src2);
      }
      ru_put(s_buf, lbase + q, ((r >> 11) & 15u) + 1u, v);
      if (two) ru_put(s_buf, lbase + q2, ((r2 >> 11) & 15u) + 1u, v2);
    }
    rs_lds_order();
    // raw stretch k+2 requested only now: the far reads above never wait behind it in vmcnt
    // order, and the ordered rounds below (no global access) cover its latency
    load_raw(k + 2, ra0, ra1);
#ifdef HBAM_PROF
    p_pre += PROF_CLK() - q1;
#endif
    // ---- ordered units: dataflow rounds (a unit is ready when no byte of its source is still
    // to be written by an earlier unit)
    if (nord && nord <= 64u) {
      // one unit per lane: dependencies as unit-index ranges (destinations are disjoint and in
      // index order): a round is a compare against the wave's done mask plus the copies
      const bool mine = lane < nord;
      const uint32_t r = mine ? s_unit[RU_CAP - 1u - lane] : 0u;
      const uint32_t q = s0 + (r & 2047u), n = ((r >> 11) & 15u) + 1u, dist = ((r >> 15) & 0x7fffu) + 1u;
      const bool per = (r >> 30) & 1u;
      const uint32_t a = q - dist, e = per ? q : a + n;
      const uint32_t vp = mine ? q : 0xffffffffu, ve = mine ? q + n : 0xffffffffu;
      uint32_t lo = 0, hi = 0;
#pragma unroll
      for (uint32_t step = 32; step; step >>= 1) {
        if (__shfl(ve, lo + step - 1u) <= a) lo += step;
        if (__shfl(vp, hi + step - 1u) < e) hi += step;
      }
      const uint64_t need = (hi > lo && mine) ? ((hi - lo == 64u ? ~0ull : ((1ull << (hi - lo)) - 1ull)) << lo) : 0ull;
      uint64_t done = ~__ballot(mine);
      // the round's bookkeeping as wave-uniform masks: one compare + ballot gives the ready set,
      // the copy runs under one exec mask with all five writes issued (no per-dword branches);
      // against per-lane ready/fin flags: ordered phase 600k -> 555k cycles per block, resolve
      // 15.63 -> 15.44 ms at 5 GB (profiles/r05/ab/resolve_sround_5g.txt)
      const uint64_t lbit = 1ull << lane;
      for (;;) {
        const uint64_t rb = __ballot((done & need) == need) & ~done;
        if (rb == 0ull) {  // validated descriptors always make progress: corrupt
          if (lane == 0) status[b] = INF_DATA;
          return;
        }
        if (rb & lbit) ru_copy<true>(s_buf, lbase + q, n, dist, per, s_sel);
        rs_lds_order();
        done |= rb;
#ifdef HBAM_PROF
        ++n_bat;
#endif
        if (done == ~0ull) break;
      }
    } else if (nord) {
      // more than 64: a pending-byte bitmap over the stretch (+ spill); unit lane + 64 t
      for (uint32_t w = lane; w < RS_PW; w += 64) s_pend[w] = 0u;
      rs_wave_sync();
      const uint32_t mine = nord > lane ? (nord - lane + 63u) / 64u : 0u;
      uint32_t live = mine >= 32u ? ~0u : (1u << mine) - 1u;
#pragma unroll 1
      for (uint32_t t = 0; t < mine; ++t) {
        const uint32_t r = s_unit[RU_CAP - 1u - (lane + 64u * t)];
        rs_bits(s_pend, r & 2047u, ((r >> 11) & 15u) + 1u, true);
      }
      rs_lds_order();
      auto is_ready = [&](uint32_t r) {
        const uint32_t q = s0 + (r & 2047u), n = ((r >> 11) & 15u) + 1u, dist = ((r >> 15) & 0x7fffu) + 1u;
        const uint32_t a = q - dist, e = ((r >> 30) & 1u) ? q : a + n;
        const uint32_t lo2 = a > s0 ? a - s0 : 0u;  // bytes before the stretch are final
        return e <= s0 + lo2 || !rs_any_bit(s_pend, lo2, e - s0);
      };
      for (;;) {
        uint32_t ready = 0;
#pragma unroll 1
        for (uint32_t t = 0; t < mine; ++t)
          if ((live >> t & 1u) && is_ready(s_unit[RU_CAP - 1u - (lane + 64u * t)])) ready |= 1u << t;
        rs_lds_order();
#pragma unroll 1
        for (uint32_t t = 0; t < mine; ++t)
          if (ready >> t & 1u) {
            const uint32_t r = s_unit[RU_CAP - 1u - (lane + 64u * t)];
            const uint32_t rel = r & 2047u, n = ((r >> 11) & 15u) + 1u, dist = ((r >> 15) & 0x7fffu) + 1u;
            ru_copy(s_buf, lbase + s0 + rel, n, dist, (r >> 30) & 1u, s_sel);
            rs_bits(s_pend, rel, n, false);
          }
        live &= ~ready;
        if (!__any(live != 0u)) break;
        if (!__any(ready != 0u)) {  // validated descriptors always make progress: corrupt
          if (lane == 0) status[b] = INF_DATA;
          return;
        }
        rs_lds_order();
      }
    }
    if ((tail0 & 0x80000000u) && (tail0 & 0xffffu) / RS_S == k && lane == 0) {
      // final match shorter than 3 bytes (the output filled up inside it); last token
      const uint32_t p = tail0 & 0xffffu, n = (tail0 >> 16) & 0x7fffu;
      uint32_t d = tails[2 * (uint64_t)b + 1];
      bool tail_bad = false;
      if (d == 0u || d > p || p + n > isize) {  // corrupt tail token: no copy from outside
        status[b] = INF_DATA;
        d = 1u;
        tail_bad = true;
      }
      uint32_t jj = 0;
      for (uint32_t t = 0; t < n && !tail_bad; ++t) {
        const uint32_t x = p - d + jj;
        s_buf[lbase + p + t] = (x + RS_W + a0 >= s0) ? s_buf[lbase + x] : ubuf[base + x];
        jj = (jj + 1u == d) ? 0u : jj + 1u;
      }
    }
    __syncthreads();
#ifdef HBAM_PROF
    const uint64_t q2 = PROF_CLK();
    p_bat += q2 - q1;
#endif
    // ---- write back stretch k, slide the window by RS_S (as k_resolve)
    uint4 wbv[RS_C];
#pragma unroll
    for (uint32_t h2 = 0; h2 < RS_C; ++h2) wbv[h2] = *(const uint4*)(s_buf + RS_W + 1024u * h2 + 16u * lane);
#pragma unroll
    for (uint32_t o = 16u * lane; o < RS_W + RS_S; o += 1024u) *(uint4*)(s_buf + o) = *(const uint4*)(s_buf + RS_S + o);
    *(uint4*)(s_buf + RS_W + RS_S + 16u * lane) = ra0;
    if (RS_C == 2) *(uint4*)(s_buf + RS_W + RS_S + 1024 + 16u * lane) = ra1;
#pragma unroll
    for (uint32_t h2 = 0; h2 < RS_C; ++h2) rs_write_back(ubuf, abase + s0 + 1024u * h2 + 16u * lane, base, aend, wbv[h2]);
    __syncthreads();
#ifdef HBAM_PROF
    p_wb += PROF_CLK() - q2;
#endif
  }
#ifdef HBAM_PROF
  if (g_prof && lane == 0) {
    unsigned long long* g = g_prof + 32 * (uint64_t)b;
    g[0] = pr0;
    g[1] = PROF_RT();
    g[2] = PROF_CLK() - pc0;
    g[3] = p_st;
    g[4] = p_desc;
    g[5] = p_bat;
    g[12] = p_pre;
    g[13] = p_wb;
    g[6] = n_bat;
    g[7] = n_m;
  }
#endif
}
