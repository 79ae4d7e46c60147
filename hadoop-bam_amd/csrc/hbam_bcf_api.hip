// hbam_bcf_api.hip — C-ABI of the BCF read path, included at the end of
// hbam_capi.hip (it uses that file's buffers, block chain, inflate and guess-window helpers).
//
//   hbam_bcf_parse_header      BCF2Codec.readHeader on the file's first bytes (BGZF inflated on
//                              the device): contig / sample / string-dictionary counts.
//   hbam_guess_bcf_windows     BCFSplitGuesser.guessNextBCFRecordStart per guess window
//                              (k_guess_bcf over the BAM guesser's window block cache).
//   hbam_bcf_decode_split      BCFRecordReader over one split: FileVirtualSplit (BGZF) or
//                              FileSplit (uncompressed), columns on the device.
// Parity: oracle/hbam_oracle_bcf.c (the record decode is a restated subset of htsjdk's
// BCF2Codec: parity unpinned).

namespace {

// ---- header --------------------------------------------------------------------------------
// BCF2Codec.readHeader over uncompressed stream bytes (same rules as or_bcf_read_header)
int bcf_header_text(const uint8_t* u, uint64_t n, hbam_bcf_header* h) {
  if (n < 9) return HBAM_EMORE;
  if (!(u[0] == 'B' && u[1] == 'C' && u[2] == 'F' && u[3] == 2 && u[4] >= 1)) return HBAM_ETRIBBLE;
  const int32_t lt = (int32_t)rd32(u + 5);
  if (lt <= 0) return HBAM_ETRIBBLE;
  if ((uint64_t)lt + 9 > n) return HBAM_EMORE;
  const char* t = (const char*)u + 9;
  const char* te = t + lt;
  int32_t nc = 0, ns = 0;
  std::vector<std::string> ids;
  auto starts = [](const char* s, const char* e, const char* p) {
    const size_t k = strlen(p);
    return (size_t)(e - s) >= k && memcmp(s, p, k) == 0;
  };
  for (const char* l = t; l < te;) {
    const char* le = (const char*)memchr(l, '\n', (size_t)(te - l));
    if (!le) le = te;
    if (starts(l, le, "##contig=<")) {
      ++nc;
    } else if (starts(l, le, "##FILTER=<") || starts(l, le, "##INFO=<") || starts(l, le, "##FORMAT=<")) {
      const char* id = nullptr;
      for (const char* q = l + 1; q + 3 < le; ++q)
        if ((q[-1] == '<' || q[-1] == ',') && memcmp(q, "ID=", 3) == 0) { id = q + 3; break; }
      if (id) {
        const char* ie = id;
        while (ie < le && *ie != ',' && *ie != '>') ++ie;
        std::string s(id, (size_t)(ie - id));
        if (s != "PASS" && std::find(ids.begin(), ids.end(), s) == ids.end()) ids.push_back(s);
      }
    } else if (starts(l, le, "#CHROM")) {
      int32_t cols = 1;
      for (const char* q = l; q < le; ++q) cols += *q == '\t';
      ns = cols > 9 ? cols - 9 : 0;
    }
    l = le + 1;
  }
  if (nc == 0) return HBAM_ETRIBBLE;  // "Didn't find any contig lines in BCF2 file header"
  h->n_contig = nc;
  h->n_sample = ns;
  h->n_dict = 1 + (int32_t)ids.size();  // PASS first (BCF2Utils.makeDictionary)
  h->header_len = (uint64_t)lt + 9;
  return HBAM_OK;
}

bool bgzf_magic(const uint8_t* b, uint64_t n) {  // BlockCompressedInputStream.isValidFile
  return n >= 18 && b[0] == 0x1f && b[1] == 0x8b && b[2] == 8 && b[3] == 4 && b[10] == 6 && b[11] == 0 &&
         b[12] == 'B' && b[13] == 'C' && b[14] == 2 && b[15] == 0;
}

// ---- the stream a BGZF BCF split reads ------------------------------------------------------
// BCFRecordReader wraps the BlockCompressedInputStream in a BGZFLimitingStream
// (BCFRecordReader.java:177-237) under tribble's PositionalBufferedStream (512,000-byte fills).
// This replays those reads over the block table (no data needed: only sizes, the failing block
// and the chain's end): z = the stream position (ubuf offset) where the reader's stream ends,
// code = HBAM_OK for a clean end of stream, else the exception of the fill that starts at z.
struct BcfBlocks {
  const std::vector<BlockRec>* blk;
  uint64_t comp_base, nb, fb;
  int32_t fb_code, end_code;
};
int bcf_stream_end(const BcfBlocks& B, uint64_t k0, uint32_t off0, uint64_t r0, uint64_t v_end, uint64_t* z,
                   int32_t* code) {
  const std::vector<BlockRec>& blk = *B.blk;
  uint64_t k = k0;
  uint32_t off = off0;
  auto isz = [&](uint64_t j) -> uint32_t { return j < B.nb ? blk[j].isize : 0u; };
  auto tell = [&]() -> uint64_t {  // getFilePointer()
    if (k >= B.nb) return (B.comp_base + blk[B.nb - 1].coff + blk[B.nb - 1].clen) << 16;
    if (off == isz(k)) return (B.comp_base + blk[k].coff + blk[k].clen) << 16;
    return (B.comp_base + blk[k].coff) << 16 | off;
  };
  // BlockCompressedInputStream.read(buf, off, n): bytes, -1, or an exception (*err)
  auto bread = [&](int32_t n, int32_t* err) -> int32_t {
    int32_t done = 0;
    while (n > 0) {
      if (k >= B.nb || off == isz(k)) {  // available(): readBlock
        const uint64_t nk = k >= B.nb ? B.nb : k + 1;
        if (nk >= B.nb) {
          if (B.end_code != HBAM_EEOF) { *err = B.end_code; return 0; }
          k = B.nb;  // count == 0: an empty current block
          off = 0;
          return done ? done : -1;
        }
        if (nk == B.fb) { *err = B.fb_code; return 0; }
        k = nk;
        off = 0;
        if (isz(k) == 0) return done ? done : -1;  // an empty block: available() == 0
      }
      const int32_t c = (int32_t)std::min<uint32_t>((uint32_t)n, isz(k) - off);
      off += (uint32_t)c;
      n -= c;
      done += c;
    }
    return done;
  };
  const int32_t last_len = (int32_t)(v_end & 0xffff);
  uint64_t fill_at = r0;
  for (;;) {
    int32_t total = 0, len = 512000, err = HBAM_OK;
    bool minus1 = false, full = false;
    uint64_t virt;
    while (((virt = tell()) >> 16) != (v_end >> 16)) {
      const int32_t want = std::min(len, last_len);
      if (want <= 0) return HBAM_EUNSUPPORTED;  // read(buf, off, 0) forever in the reference
      const int32_t r = bread(want, &err);
      if (err) break;
      if (r == -1) { minus1 = true; break; }
      total += r;
      len -= r;
      if (len == 0) { full = true; break; }
    }
    if (!err && !minus1 && !full) {  // in the block at vEnd's offset (:224-235)
      const int32_t lim = (int32_t)(tell() & 0xffff) - last_len;
      if (lim < len) len = lim;
      while (len > 0) {
        const int32_t r = bread(len, &err);
        if (err) break;
        if (r == -1) break;
        total += r;
        len -= r;
      }
    }
    if (err) { *z = fill_at; *code = err; return HBAM_OK; }
    if (total == 0) { *z = fill_at; *code = HBAM_OK; return HBAM_OK; }  // -1: end of stream
    fill_at += (uint64_t)total;
  }
}

int bcf_cols(hbam_ctx* c, uint64_t n, BcfCols* k) {
  uint8_t* base;
  int rc;
  const uint64_t m = n + 1;
  if ((rc = ensure(c, B_BCF_COLS, m * (9 * 4 + 2 * 8) + 64, &base))) return rc;
  int64_t* q8 = (int64_t*)base;
  k->key = q8;
  k->rel = q8 + m;
  int32_t* q4 = (int32_t*)(q8 + 2 * m);
  k->status = q4;
  k->l_shared = q4 + m;
  k->l_indiv = q4 + 2 * m;
  k->chrom = q4 + 3 * m;
  k->pos = q4 + 4 * m;
  k->rlen = q4 + 5 * m;
  k->qual = (uint32_t*)(q4 + 6 * m);
  k->n_allele_info = q4 + 7 * m;
  k->n_fmt_sample = q4 + 8 * m;
  return HBAM_OK;
}

}  // namespace

extern "C" int hbam_bcf_parse_header(hbam_ctx* c, const uint8_t* file, uint64_t len, hbam_bcf_header* out) {
  if (!c || !file || !out) return HBAM_EINVAL;
  memset(out, 0, sizeof *out);
  HIPCHK(c, hipSetDevice(c->device));
  if (!bgzf_magic(file, len)) {
    out->bgzf = 0;
    int rc = bcf_header_text(file, len, out);
    if (rc == HBAM_OK) out->first_voffset = out->header_len;
    return rc;
  }
  out->bgzf = 1;
  // inflate the leading blocks on the device until the header text is complete
  std::vector<uint8_t> u;
  std::vector<uint64_t> ustart;  // stream position of each block, for first_voffset
  std::vector<uint64_t> coffs;
  uint64_t p = 0;
  const uint8_t* d;
  int rc = stage_comp(c, file, 0, len, &d);
  if (rc) return rc;
  for (;;) {
    if (p + 18 > len) return HBAM_EMORE;
    const uint32_t bl = (uint32_t)rd16(file + p + 16) + 1u;
    if (p + bl > len) return HBAM_EMORE;
    const uint32_t isize = (uint32_t)rd32(file + p + bl - 4);
    if (bl < 26 || isize > 65536u) return HBAM_EFORMAT;
    BlockRec r{p, bl, isize, (uint32_t)rd32(file + p + bl - 8), 0};
    BlockRec* blk;
    uint64_t* uo;
    uint8_t* ub;
    int32_t* st;
    uint32_t* crc;
    if ((rc = ensure(c, B_BLK, 2, &blk)) || (rc = ensure(c, B_UOFF, 2, &uo)) ||
        (rc = ensure(c, B_UBUF, 65536 + UBUF_SLACK, &ub)) || (rc = ensure(c, B_INFST, 2, &st)) ||
        (rc = ensure(c, B_CRC, 2, &crc)))
      return rc;
    const uint64_t zero = 0;
    HIPCHK(c, hipMemcpyAsync(blk, &r, sizeof r, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(uo, &zero, 8, hipMemcpyHostToDevice, c->stream));
    if ((rc = inflate_blocks(c, d, blk, 1, uo, ub, st, false, crc))) return rc;
    int32_t s;
    HIPCHK(c, copy_sync(c, &s, st, 4, hipMemcpyDeviceToHost));
    if (s != INF_OK) return s == INF_DATA ? HBAM_EDATA : HBAM_EFORMAT;
    const size_t at = u.size();
    u.resize(at + isize);
    if (isize) HIPCHK(c, copy_sync(c, u.data() + at, ub, isize, hipMemcpyDeviceToHost));
    ustart.push_back(at);
    coffs.push_back(p);
    p += bl;
    rc = bcf_header_text(u.data(), u.size(), out);
    if (rc != HBAM_EMORE) break;
  }
  out->bgzf = 1;
  if (rc) return rc;
  // virtual offset of the first record (getFilePointer() after the header): the block holding
  // stream byte header_len, or the next block's start when the header ends with a block
  out->first_voffset = p << 16;
  for (size_t j = 0; j < ustart.size(); ++j) {
    const uint64_t e = j + 1 < ustart.size() ? ustart[j + 1] : u.size();
    if (out->header_len < e) {
      out->first_voffset = coffs[j] << 16 | (out->header_len - ustart[j]);
      break;
    }
  }
  return HBAM_OK;
}

extern "C" uint64_t hbam_guess_bcf_window_len(uint64_t file_len, int64_t beg, int64_t end, int bgzf) {
  return window_len(file_len, beg, end, bgzf ? BCF_BGZF_WINDOW : BCF_UNCOMP_NEEDED);
}

extern "C" int hbam_guess_bcf_windows(hbam_ctx* c, const uint8_t* windows, int on_device, const uint64_t* win_off,
                                      uint64_t file_len, const int64_t* beg, const int64_t* end, uint64_t k,
                                      const hbam_bcf_header* h, int64_t* out, int32_t* err) {
  if (!c || !h || (k && (!windows || !win_off || !beg || !end || !out || !err))) return HBAM_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  if (k == 0) return HBAM_OK;
  const int bgzf = h->bgzf ? 1 : 0;
  std::vector<uint64_t> wp;
  std::vector<int64_t> wl;
  int rc = caller_windows(c, windows, on_device, win_off, file_len, beg, end, k,
                          bgzf ? BCF_BGZF_WINDOW : BCF_UNCOMP_NEEDED, &wp, &wl);
  if (rc) return rc;
  const BcfHdr bh{h->n_contig, h->n_sample, h->n_dict};
  HIPCHK(c, hipEventRecord(c->ev[9], c->stream));
  const uint64_t batch = 1024;  // 3 x 64 KiB of inflate scratch per guess
  for (uint64_t g0 = 0; g0 < k; g0 += batch) {
    const uint64_t kb = std::min(batch, k - g0);
    GuessWork w;
    uint8_t* scratch;
    if ((rc = guess_work(c, kb, &w))) return rc;
    if ((rc = ensure(c, B_BCF_SCRATCH, kb * 3 * 65536 + 64, &scratch))) return rc;
    HIPCHK(c, hipMemcpyAsync(w.beg, beg + g0, kb * 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(w.end, end + g0, kb * 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(w.wptr, wp.data() + g0, kb * 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(w.wlen, wl.data() + g0, kb * 8, hipMemcpyHostToDevice, c->stream));
    GuessCache gc;
    if (bgzf && (rc = build_guess_cache(c, w, kb, &gc))) return rc;
    k_guess_bcf<<<grid_for(kb, GUESS_WG), GUESS_WG, 0, c->stream>>>(
        w.wptr, w.wlen, w.beg, w.end, (uint32_t)kb, bgzf, bh, scratch, w.lens, w.out, w.err, gc.cn, gc.cbase,
        gc.cpos, gc.cblk, gc.cuoff, gc.cubuf, gc.cst, gc.ccrc);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemcpyAsync(out + g0, w.out, kb * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(err + g0, w.err, kb * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
  }
  HIPCHK(c, hipEventRecord(c->ev[10], c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->timing = hbam_timing{};
  c->timing.total_ms = ev_ms(c, 9, 10);
  return HBAM_OK;
}

extern "C" int hbam_bcf_decode_split(hbam_ctx* c, const uint8_t* comp, int on_device, uint64_t comp_base,
                                     uint64_t comp_len, uint64_t file_len, const hbam_bcf_header* h,
                                     uint64_t v_start, uint64_t v_end, hbam_bcf_columns* out) {
  if (!c || !comp || !h || !out) return HBAM_EINVAL;
  memset(out, 0, sizeof *out);
  HIPCHK(c, hipSetDevice(c->device));
  if (comp_base + comp_len > file_len) return set_err(c, HBAM_EINVAL, "window past the end of the file");
  const bool window_is_file_end = comp_base + comp_len == file_len;
  if (!h->bgzf && !window_is_file_end)
    return set_err(c, HBAM_EINVAL, "an uncompressed BCF split reads to the end of the file: the window must reach it");
  c->timing = hbam_timing{};
  const uint8_t* d;
  int rc = stage_comp(c, comp, on_device, comp_len, &d);
  if (rc) return rc;
  const BcfHdr bh{h->n_contig, h->n_sample, h->n_dict};
  HIPCHK(c, hipEventRecord(c->ev[0], c->stream));
  const uint8_t* ub;     // the record stream
  uint64_t ulen;         // its bytes
  const uint64_t* uo;    // walk segments
  uint64_t wb;           // segments
  uint64_t r0, z, limit = ~0ULL, rel_base = 0;
  int64_t rel_add = 0;
  int32_t z_code = HBAM_OK;
  if (h->bgzf) {
    const uint64_t coff_s = v_start >> 16;
    const uint32_t uoff_s = (uint32_t)(v_start & 0xffff);
    if (coff_s < comp_base || coff_s > comp_base + comp_len)
      return set_err(c, HBAM_EINVAL, "v_start outside the compressed window");
    Chain ch;
    if ((rc = build_chain(c, d, comp_len, coff_s - comp_base, window_is_file_end, &ch))) return rc;
    const uint64_t nb = ch.nb;
    if (nb == 0) {  // initialize(): bci.seek(virtualStart) fails, or an empty stream
      if (ch.end_code == HBAM_EMORE) {
        out->status = HBAM_EMORE;
        return HBAM_OK;
      }
      if (ch.end_code == HBAM_EEOF) {
        out->status = uoff_s != 0 ? HBAM_EIO : HBAM_OK;
        return HBAM_OK;
      }
      out->status = ch.end_code == HBAM_ERUNTIMEIO ? HBAM_EIO : ch.end_code;
      return HBAM_OK;
    }
    BlockRec* blk = (BlockRec*)c->bufs[B_BLK].p;
    uint32_t* isz;
    uint64_t* uoff;
    uint64_t* small;
    if ((rc = ensure(c, B_ISZ32, nb + 1, &isz)) || (rc = ensure(c, B_UOFF, nb + 1, &uoff)) ||
        (rc = ensure(c, B_SMALL, 16, &small)))
      return rc;
    HIPCHK(c, hipMemsetAsync(small, 0xff, 8 * 8, c->stream));
    k_isize32<<<grid_for(nb, 256), 256, 0, c->stream>>>(blk, nb, isz, (uint32_t*)small);
    uint64_t utotal = 0;
    if ((rc = scan_exclusive<uint32_t>(c, isz, nb, uoff, &utotal))) return rc;
    std::vector<BlockRec> hb(nb);
    std::vector<uint64_t> hu(nb + 1);
    HIPCHK(c, hipMemcpyAsync(hb.data(), blk, nb * sizeof(BlockRec), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(hu.data(), uoff, (nb + 1) * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->pinned_small, small, 16, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const uint32_t bigi = (uint32_t)(c->pinned_small[0] & 0xffffffffu);
    // bci.seek(virtualStart): the block at coff_s, or the next one when it is empty
    const uint64_t sblk = hb[0].isize == 0 ? 1 : 0;
    // Where BGZFLimitingStream stops (the replay needs block sizes only): with every block assumed
    // to inflate, the stream ends at z0; only the blocks up to z0's (and one more) are inflated, so
    // a split costs its own blocks, not the rest of the file.  A block failing before
    // that point ends the stream earlier: the replay runs again with it (z only moves back).
    uint64_t z0 = 0;
    int32_t zc0 = HBAM_OK;
    if (sblk < nb) {
      r0 = hu[sblk] + uoff_s;
      const BcfBlocks B0{&hb, comp_base, nb, nb, HBAM_OK, ch.end_code};
      if ((rc = bcf_stream_end(B0, sblk, uoff_s, r0, v_end, &z0, &zc0)))
        return set_err(c, rc, "BGZFLimitingStream with vEnd & 0xffff == 0 never returns");
      if (zc0 == HBAM_EMORE) {  // the stream runs past the window: the caller passes a longer one
        out->status = HBAM_EMORE;
        return HBAM_OK;
      }
    }
    uint64_t nbi = nb;  // blocks inflated
    if (sblk < nb) {
      uint64_t zb = sblk;
      while (zb + 1 < nb && hu[zb + 1] <= z0) ++zb;
      nbi = std::min<uint64_t>(nb, zb + 2);
    } else {
      nbi = std::min<uint64_t>(nb, 2);
    }
    const uint64_t ui = hu[nbi];
    uint8_t* ubw;
    int32_t* st;
    uint32_t* crc;
    if ((rc = ensure(c, B_UBUF, ui + UBUF_SLACK, &ubw)) || (rc = ensure(c, B_INFST, nbi + 1, &st)) ||
        (rc = ensure(c, B_CRC, nbi + 1, &crc)))
      return rc;
    if ((rc = inflate_blocks(c, d, blk, nbi, uoff, ubw, st, false, crc))) return rc;
    unsigned long long* first_bad = (unsigned long long*)small + 1;
    k_first_bad_block<<<grid_for(nbi, 256), 256, 0, c->stream>>>(st, crc, blk, nbi, 0, first_bad);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemcpyAsync(c->pinned_small, small, 16, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    uint64_t fb = c->pinned_small[1];
    int32_t fb_code = HBAM_EEOF;
    if (fb != ~0ULL) {
      int32_t s;
      HIPCHK(c, copy_sync(c, &s, st + fb, 4, hipMemcpyDeviceToHost));
      fb_code = (s == INF_DATA) ? HBAM_EDATA : HBAM_EFORMAT;
    }
    if (bigi != 0xffffffffu && bigi < nbi && (fb == ~0ULL || bigi < fb)) {
      fb = bigi;
      fb_code = HBAM_EUNSUPPORTED;
    }
    if (fb == ~0ULL) fb = nb;
    if (fb == 0) { out->status = fb_code; return HBAM_OK; }
    if (sblk >= nb) {
      if (ch.end_code != HBAM_EEOF) { out->status = ch.end_code == HBAM_ERUNTIMEIO ? HBAM_EIO : ch.end_code; return HBAM_OK; }
      out->status = uoff_s != 0 ? HBAM_EIO : HBAM_OK;
      return HBAM_OK;
    }
    if (fb == sblk) { out->status = fb_code; return HBAM_OK; }
    {
      const BlockRec& bs = hb[sblk];
      const uint64_t after = comp_base + bs.coff + bs.clen;
      const bool eof = (after == file_len) || (file_len - after == 28);
      if (uoff_s > bs.isize || (uoff_s == bs.isize && !eof)) { out->status = HBAM_EIO; return HBAM_OK; }
    }
    z = z0;
    z_code = zc0;
    if (fb < nb) {
      const BcfBlocks B{&hb, comp_base, nb, fb, fb_code, ch.end_code};
      if ((rc = bcf_stream_end(B, sblk, uoff_s, r0, v_end, &z, &z_code)))
        return set_err(c, rc, "BGZFLimitingStream with vEnd & 0xffff == 0 never returns");
    }
    ub = ubw;
    ulen = ui;
    uo = uoff + sblk;
    wb = nbi - sblk;
    rel_base = r0;
  } else {
    // FileSplit: the header is read through the stream first, then skip(start - position)
    const uint64_t start = std::max<uint64_t>(v_start, h->header_len);
    if (start < comp_base) return set_err(c, HBAM_EINVAL, "split start before the window");
    ub = d;
    ulen = comp_len;
    r0 = std::min<uint64_t>(start - comp_base, comp_len);
    z = comp_len;
    limit = v_start + v_end >= comp_base ? v_start + v_end - comp_base : 0;
    rel_add = (int64_t)comp_base;
    const uint32_t nseg = (uint32_t)((comp_len + 65535) >> 16);
    uint64_t* seg;
    if ((rc = ensure(c, B_UOFF, (uint64_t)nseg + 2, &seg))) return rc;
    k_raw_segments<<<grid_for((uint64_t)nseg + 1, 256), 256, 0, c->stream>>>(comp_len, nseg, seg);
    HIPCHK(c, hipGetLastError());
    // walk from the segment holding r0
    const uint64_t s0 = r0 >> 16;
    uo = seg + s0;
    wb = nseg > s0 ? nseg - s0 : 0;
  }
  HIPCHK(c, hipEventRecord(c->ev[4], c->stream));
  // ---- record chain (the BAM walk with BCF2 framing)
  uint64_t nrec = 0, exit_last = r0;
  uint64_t* rec_off = nullptr;
  if (wb && r0 < ulen) {
    uint64_t *entry, *exitp, *rbase;
    uint16_t* rel;
    uint32_t *count, *badlist, *nbad_d;
    uint8_t* mark;
    uint64_t* small;
    if ((rc = ensure(c, B_ENTRY, wb + 1, &entry)) || (rc = ensure(c, B_EXIT, wb + 1, &exitp)) ||
        (rc = ensure(c, B_REL, wb * WALK_CAP, &rel)) || (rc = ensure(c, B_COUNT, wb + 1, &count)) ||
        (rc = ensure(c, B_RECBASE, wb + 1, &rbase)) || (rc = ensure(c, B_BADLIST, wb + 1, &badlist)) ||
        (rc = ensure(c, B_MARK, wb + 1, &mark)) || (rc = ensure(c, B_SMALL, 16, &small)))
      return rc;
    const BcfFmt fmt{bh};
    const uint64_t hard_end = z;
    if (wb > 1) k_block_entry<<<(uint32_t)(wb - 1), 64, 0, c->stream>>>(ub, uo, (uint32_t)wb, hard_end, fmt, entry);
    k_block_walk<<<grid_for(wb, 64), 64, 0, c->stream>>>(ub, uo, (uint32_t)wb, r0, hard_end, fmt, entry, rel, count,
                                                         exitp);
    nbad_d = (uint32_t*)(small + 5);
    HIPCHK(c, hipMemsetAsync(nbad_d, 0, 4, c->stream));
    HIPCHK(c, hipMemsetAsync(mark, 0, 1, c->stream));
    if (wb > 1)
      k_stitch_check<<<grid_for(wb - 1, 256), 256, 0, c->stream>>>(entry, exitp, (uint32_t)wb, nbad_d, badlist,
                                                                   (uint32_t)wb, mark);
    uint32_t nbad = 0;
    HIPCHK(c, hipMemcpyAsync(&nbad, nbad_d, 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (nbad) {
      k_chain_fix_par<<<grid_for(nbad, 64), 64, 0, c->stream>>>(ub, uo, (uint32_t)wb, hard_end, fmt, entry, rel,
                                                                 count, exitp, badlist, nbad, mark);
      HIPCHK(c, hipMemsetAsync(nbad_d, 0, 4, c->stream));
      k_stitch_check<<<grid_for(wb - 1, 256), 256, 0, c->stream>>>(entry, exitp, (uint32_t)wb, nbad_d, badlist,
                                                                   (uint32_t)wb, nullptr);
      HIPCHK(c, hipMemcpyAsync(&nbad, nbad_d, 4, hipMemcpyDeviceToHost, c->stream));
      HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    if (nbad) {
      std::vector<uint32_t> bl(nbad);
      HIPCHK(c, copy_sync(c, bl.data(), badlist, nbad * 4, hipMemcpyDeviceToHost));
      std::sort(bl.begin(), bl.end());
      HIPCHK(c, copy_sync(c, badlist, bl.data(), nbad * 4, hipMemcpyHostToDevice));
      k_chain_fix<<<1, 64, 0, c->stream>>>(ub, uo, (uint32_t)wb, hard_end, fmt, entry, rel, count, exitp, badlist,
                                           nbad);
      HIPCHK(c, hipGetLastError());
    }
    if ((rc = scan_exclusive<uint32_t>(c, count, wb, rbase, &nrec))) return rc;
    HIPCHK(c, copy_sync(c, &exit_last, exitp + (wb - 1), 8, hipMemcpyDeviceToHost));
    if ((rc = ensure(c, B_RECOFF, nrec + 1, &rec_off))) return rc;
    k_emit_rec_off<<<(uint32_t)wb, 256, 0, c->stream>>>(uo, (uint32_t)wb, rel, count, rbase, rec_off);
    HIPCHK(c, hipGetLastError());
  }
  HIPCHK(c, hipEventRecord(c->ev[5], c->stream));
  // ---- per record: nextKeyValue
  BcfCols bc;
  if ((rc = bcf_cols(c, nrec, &bc))) return rc;
  uint64_t* small;
  if ((rc = ensure(c, B_SMALL, 16, &small))) return rc;
  unsigned long long* first_stop = (unsigned long long*)small + 6;
  HIPCHK(c, hipMemsetAsync(first_stop, 0xff, 8, c->stream));
  if (nrec)
    k_bcf_decode<<<grid_for(nrec, 256), 256, 0, c->stream>>>(ub, nrec, rec_off, z, z_code, limit, rel_base,
                                                              rel_add, bh, bc, first_stop);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipEventRecord(c->ev[6], c->stream));
  uint64_t fs;
  HIPCHK(c, hipMemcpyAsync(&fs, first_stop, 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  uint64_t n_final = std::min<uint64_t>(fs, nrec);
  int32_t status = HBAM_OK;
  if (fs < nrec) {
    int32_t s;
    HIPCHK(c, copy_sync(c, &s, bc.status + fs, 4, hipMemcpyDeviceToHost));
    if (s < 0) status = s;
  } else if (z_code != HBAM_OK && exit_last == z) {
    status = z_code;  // the next peek() needs the fill that fails
  } else if (z_code != HBAM_OK && nrec == 0 && r0 >= z) {
    status = z_code;
  }
  out->n_records = n_final;
  out->status = status;
  out->err_record = n_final;
  out->rel = bc.rel;
  out->rec_off = rec_off;
  out->data = (uint8_t*)ub;
  out->data_len = ulen;
  out->key = bc.key;
  out->l_shared = bc.l_shared;
  out->l_indiv = bc.l_indiv;
  out->chrom = bc.chrom;
  out->pos = bc.pos;
  out->rlen = bc.rlen;
  out->qual = bc.qual;
  out->n_allele_info = bc.n_allele_info;
  out->n_fmt_sample = bc.n_fmt_sample;
  c->timing.walk_ms = ev_ms(c, 4, 5);
  c->timing.decode_ms = ev_ms(c, 5, 6);
  c->timing.total_ms = ev_ms(c, 0, 6);
  c->timing.ubuf_bytes = ulen;
  c->timing.n_records = n_final;
  return HBAM_OK;
}
