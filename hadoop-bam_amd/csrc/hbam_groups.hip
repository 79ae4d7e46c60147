// hbam_groups.hip — multi-input Sort: Utils.correctSAMRecordForMerging's program-group and
// read-group rewrite (cli/Utils.java:314-324) over a decoded split, on the device.
//
// When SamFileHeaderMerger reports ID collisions among the inputs' @PG (or @RG) records, every
// record of input h that carries a PG (or RG) tag gets setAttribute(tag, merger.getProgramGroupId(h,
// value)).  The reference looks RG values up in the PROGRAM-group table too (:322), so an RG value
// becomes the translated PG id of the same string, or — not a PG id of h — null, which removes the
// tag; an input whose header has no @PG record has no table at all, and the lookup throws
// NullPointerException.  `(String) r.getAttribute(tag)` throws ClassCastException for a tag that
// is not a string ('Z').  A record on which setAttribute ran is re-encoded by
// SAMRecordWritable.write -> BAMRecordCodec.encode (htsjdk 1.131, restated, parity unpinned): the
// variable block is re-serialised from the decoded fields — integer tags re-typed by
// BinaryTagCodec.getIntegerType, the odd-length sequence's pad nibble zeroed, absent qualities
// written as 0xFF — and the bin written as 0 for an unplaced record; a replaced tag keeps its
// place in the attribute list, a removed one leaves it (the FixMate encoder's rule,
// hbam_consumers.hip).  One thread per record: length pass, exclusive scan, write pass.
#pragma once

namespace hbam {

// table (device copy of the host table, see include/hbam.h): per tag (PG, RG) mode u8, count u16,
// entries {u16 old_len, old bytes, i16 new_len, new bytes}
struct GrpTab {
  const uint8_t* t;
  uint32_t off[2];  // first entry of each tag
  uint32_t cnt[2];
  uint32_t mode[2];  // 0 untouched, 1 translate, 2 NullPointerException
};
constexpr uint8_t GRP_TAG[2][2] = {{'P', 'G'}, {'R', 'G'}};

// new value of (tag k, value v[0..vl)): 1 found (*nv, *nl), 0 not in the table (-> removed)
__device__ int grp_lookup(const GrpTab& g, int k, const uint8_t* v, uint32_t vl, const uint8_t** nv, int32_t* nl) {
  uint32_t o = g.off[k];
  for (uint32_t e = 0; e < g.cnt[k]; ++e) {
    const uint32_t ol = (uint32_t)g.t[o] | (uint32_t)g.t[o + 1] << 8;
    const uint8_t* ov = g.t + o + 2;
    const int32_t wl = (int16_t)((uint16_t)(g.t[o + 2 + ol] | g.t[o + 3 + ol] << 8));
    const uint8_t* wv = g.t + o + 4 + ol;
    bool eq = ol == vl;
    for (uint32_t q = 0; eq && q < vl; ++q) eq = ov[q] == v[q];
    if (eq) {
      *nv = wv;
      *nl = wl;
      return 1;
    }
    o += 4 + ol + (wl > 0 ? (uint32_t)wl : 0u);
  }
  return 0;
}

// one record: -> new payload length (dst == nullptr: length only), or -(1 + status index):
// 1 NullPointerException, 2 ClassCastException, 3 SAMFormatException
__device__ int64_t grp_encode(const uint8_t* __restrict__ r, const GrpTab& g, uint8_t* __restrict__ dst) {
  const int32_t bs = f4_ld32(r);
  const uint32_t lrn = r[12], nc = f4_ld16(r + 16);
  const int32_t lseq = f4_ld32(r + 20);
  const uint64_t ls = lseq > 0 ? (uint64_t)lseq : 0;
  const uint64_t head = 36 + lrn + 4ull * nc, sq = (ls + 1) / 2;
  const uint64_t vstart = head + sq + ls;
  if (bs < 32 || vstart > (uint64_t)bs + 4) return -4;
  const uint8_t* aux = r + vstart;
  const uint64_t aux_len = (uint64_t)bs + 4 - vstart;
  // the first occurrence of each tag (SAMRecord.getAttribute walks the list from its head)
  int64_t at[2] = {-1, -1};
  bool parsed = true;
  for (uint64_t p = 0; p < aux_len;) {
    if (aux_len - p < 3) { parsed = false; break; }
    const char ty = (char)aux[p + 2];
    const int64_t vs = f4_aux_vsize(aux + p + 3, aux_len - p - 3, ty);
    if (vs < 0 || (uint64_t)vs > aux_len - p - 3) { parsed = false; break; }
    for (int k = 0; k < 2; ++k)
      if (at[k] < 0 && aux[p] == GRP_TAG[k][0] && aux[p + 1] == GRP_TAG[k][1]) at[k] = (int64_t)p;
    p += 3 + (uint64_t)vs;
  }
  // correctSAMRecordForMerging: PG first, then RG; getAttribute decodes every attribute
  bool stale = false;
  const uint8_t* nv[2] = {nullptr, nullptr};
  int32_t nl[2] = {0, 0};
  bool edit[2] = {false, false};
  for (int k = 0; k < 2; ++k) {
    if (g.mode[k] == 0) continue;
    if (!parsed) return -4;
    if (at[k] < 0) continue;  // getAttribute == null: untouched
    const uint8_t* v = aux + at[k] + 3;
    if ((char)aux[at[k] + 2] != 'Z') return -3;  // (String) of a non-String attribute
    if (g.mode[k] == 2) return -2;               // samProgramGroupIdTranslation.get(h) == null
    const uint32_t vl = (uint32_t)f4_aux_vsize(v, aux_len - at[k] - 3, 'Z') - 1u;
    if (!grp_lookup(g, k, v, vl, &nv[k], &nl[k])) nl[k] = -1;  // get(value) == null: removed
    edit[k] = true;
    stale = true;
  }
  if (!stale) {  // the record's own bytes (SAMRecordWritable writes the unchanged binary block)
    if (dst)
      for (int64_t q = 0; q < (int64_t)bs + 4; ++q) dst[q] = r[q];
    return (int64_t)bs + 4;
  }
  uint64_t o = vstart;
  for (uint64_t p = 0; p < aux_len;) {
    const uint8_t t0 = aux[p], t1 = aux[p + 1];
    const char ty = (char)aux[p + 2];
    const int64_t vs = f4_aux_vsize(aux + p + 3, aux_len - p - 3, ty);
    int k = -1;
    for (int q = 0; q < 2; ++q)
      if (edit[q] && (int64_t)p == at[q]) k = q;
    if (k >= 0) {
      if (nl[k] >= 0) {  // setAttribute(tag, new string): in place
        if (dst) {
          dst[o] = t0;
          dst[o + 1] = t1;
          dst[o + 2] = 'Z';
          for (int32_t q = 0; q < nl[k]; ++q) dst[o + 3 + q] = nv[k][q];
          dst[o + 3 + nl[k]] = 0;
        }
        o += 4 + (uint64_t)nl[k];
      }
    } else if (ty == 'c' || ty == 'C' || ty == 's' || ty == 'S' || ty == 'i' || ty == 'I') {
      const int64_t v = f4_aux_int(aux + p + 3, ty);
      const char nt = f4_int_type(v);
      if (dst) f4_put_tag(dst + o, t0, t1, nt, v);
      o += 3 + f4_tsz(nt);
    } else {
      if (dst)
        for (uint64_t q = 0; q < 3 + (uint64_t)vs; ++q) dst[o + q] = aux[p + q];
      o += 3 + (uint64_t)vs;
    }
    p += 3 + (uint64_t)vs;
  }
  if (dst) {
    for (uint64_t q = 0; q < head; ++q) dst[q] = r[q];
    f4_st32(dst, (int32_t)(o - 4));
    if (f4_ld32(r + 4) < 0) f4_st16(dst + 14, 0);  // encode: indexBin 0 for an unplaced record
    for (uint64_t q = 0; q < sq; ++q) dst[head + q] = r[head + q];
    if (ls & 1u) dst[head + sq - 1] &= 0xf0u;  // bytesToCompressedBases: pad nibble 0
    const bool noqual = ls && r[head + sq] == 0xffu;
    for (uint64_t q = 0; q < ls; ++q) dst[head + sq + q] = noqual ? 0xffu : r[head + sq + q];
  }
  return (int64_t)o;
}

__global__ __launch_bounds__(F4_WG) void k_grp_len(const uint8_t* __restrict__ ubuf, const uint64_t* __restrict__ rec_off,
                                                   uint64_t n, GrpTab g, uint32_t* __restrict__ lens,
                                                   unsigned long long* __restrict__ first_err,
                                                   int32_t* __restrict__ err_code) {
  const uint64_t i = (uint64_t)blockIdx.x * F4_WG + threadIdx.x;
  if (i >= n) return;
  const int64_t L = grp_encode(ubuf + rec_off[i], g, nullptr);
  lens[i] = L < 0 ? 0u : (uint32_t)L;
  if (L < 0) {
    err_code[i] = (int32_t)(-L - 1);
    atomicMin(first_err, (unsigned long long)i);
  }
}

__global__ __launch_bounds__(F4_WG) void k_grp_write(const uint8_t* __restrict__ ubuf, const uint64_t* __restrict__ rec_off,
                                                     uint64_t n, GrpTab g, const uint64_t* __restrict__ ooff,
                                                     uint8_t* __restrict__ out, int32_t* __restrict__ bs_out) {
  const uint64_t i = (uint64_t)blockIdx.x * F4_WG + threadIdx.x;
  if (i >= n) return;
  grp_encode(ubuf + rec_off[i], g, out + ooff[i]);
  bs_out[i] = (int32_t)(ooff[i + 1] - ooff[i]) - 4;
}

}  // namespace hbam

extern "C" int hbam_rewrite_groups(hbam_ctx* c, hbam_columns* dv, const uint8_t* table, uint64_t table_len,
                                   int32_t* status, uint64_t* err_record) {
  if (!c || !dv || !status || !err_record || (table_len && !table)) return HBAM_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  *status = HBAM_OK;
  *err_record = ~0ull;
  // host-side parse of the table: offsets of each tag's entries
  GrpTab g{};
  uint64_t p = 0;
  for (int k = 0; k < 2; ++k) {
    if (p + 3 > table_len) return set_err(c, HBAM_EINVAL, "hbam_rewrite_groups: table truncated");
    g.mode[k] = table[p];
    g.cnt[k] = (uint32_t)table[p + 1] | (uint32_t)table[p + 2] << 8;
    if (g.mode[k] > 2) return set_err(c, HBAM_EINVAL, "hbam_rewrite_groups: mode %u", g.mode[k]);
    p += 3;
    g.off[k] = (uint32_t)p;
    for (uint32_t e = 0; e < g.cnt[k]; ++e) {
      if (p + 2 > table_len) return set_err(c, HBAM_EINVAL, "hbam_rewrite_groups: table truncated");
      const uint64_t ol = (uint64_t)table[p] | (uint64_t)table[p + 1] << 8;
      if (p + 4 + ol > table_len) return set_err(c, HBAM_EINVAL, "hbam_rewrite_groups: table truncated");
      const int32_t wl = (int16_t)((uint16_t)(table[p + 2 + ol] | table[p + 3 + ol] << 8));
      p += 4 + ol + (wl > 0 ? (uint64_t)wl : 0u);
      if (p > table_len || wl < -1) return set_err(c, HBAM_EINVAL, "hbam_rewrite_groups: bad entry");
    }
  }
  const uint64_t n = dv->n_records;
  if (n == 0 || (g.mode[0] == 0 && g.mode[1] == 0)) return HBAM_OK;
  if (n > 0xffffffffull) return set_err(c, HBAM_EINVAL, "hbam_rewrite_groups: n > 2^32-1");
  uint8_t* dtab;
  uint32_t* lens;
  uint64_t *err, *ooff;
  int32_t *codes, *bs;
  int rc;
  if ((rc = ensure(c, B_G_TAB, p + 1, &dtab)) || (rc = ensure(c, B_G_LENS, n + 1, &lens)) ||
      (rc = ensure(c, B_G_ERR, 1, &err)) || (rc = ensure(c, B_G_CODES, n + 1, &codes)) ||
      (rc = ensure(c, B_G_OOFF, n + 1, &ooff)) || (rc = ensure(c, B_G_BS, n + 1, &bs)))
    return rc;
  HIPCHK(c, hipMemcpyAsync(dtab, table, p, hipMemcpyHostToDevice, c->stream));
  g.t = dtab;
  HIPCHK(c, hipMemsetAsync(err, 0xff, 8, c->stream));
  k_grp_len<<<grid_for(n, F4_WG), F4_WG, 0, c->stream>>>(dv->ubuf, dv->rec_off, n, g, lens,
                                                         (unsigned long long*)err, codes);
  HIPCHK(c, hipGetLastError());
  uint64_t e = 0;
  HIPCHK(c, copy_sync(c, &e, err, 8, hipMemcpyDeviceToHost));
  uint64_t nkeep = n;
  if (e != ~0ull) {  // the map task fails at record e: the records before it stand
    int32_t code = 0;
    HIPCHK(c, copy_sync(c, &code, codes + e, 4, hipMemcpyDeviceToHost));
    *status = code == 1 ? HBAM_ENULL : code == 2 ? HBAM_ECLASSCAST : HBAM_EFORMAT;
    *err_record = e;
    nkeep = e;
  }
  uint64_t bytes = 0;
  if ((rc = scan_exclusive(c, lens, nkeep, ooff, &bytes))) return rc;
  uint8_t* out;
  if ((rc = ensure(c, B_G_PAY, bytes + 64, &out))) return rc;
  if (nkeep)
    k_grp_write<<<grid_for(nkeep, F4_WG), F4_WG, 0, c->stream>>>(dv->ubuf, dv->rec_off, nkeep, g, ooff, out, bs);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipStreamSynchronize(c->stream));
  dv->ubuf = out;
  dv->ubuf_len = bytes;
  dv->rec_off = ooff;
  dv->block_size = bs;
  dv->n_records = nkeep;
  return HBAM_OK;
}
