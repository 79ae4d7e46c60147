// Synthetic BAM generator (test/bench tooling, not product code).
//
// Produces deterministic, seeded, 150 bp paired-end BAM files shaped like the
// inputs SURVEY.md §8(d) specifies for the BASELINE configs:
//   * 25-contig GRCh38-like dictionary, @HD/@SQ/@RG/@PG text header;
//   * flags 99/147/83/163, ~1 % mate-unmapped pairs (73/133/137/69, the
//     unmapped mate "placed" at its mate's coordinate), ~0.5 % unplaced
//     unmapped reads (refID = -1) at the end of a sorted file;
//   * CIGAR 150M in ~90 % of reads, soft clips / 1-3 bp indels otherwise;
//   * 4-level binned qualities with 5 % noise (U/C ~ 3) or uniform Q2-Q41;
//   * aux NM:C MD:Z AS:C XS:C RG:Z MC:Z;
//   * raw DEFLATE at zlib level 5 (htsjdk's default Deflater level), BGZF
//     framing (SAM spec §4.1), records straddling blocks ("htsjdk packing") or
//     never straddling ("htslib packing"), optional empty blocks mid-file.
//
// The stream is built from independent *segments* of R records, each compressed
// on its own thread; a segment's last block is flushed short, so the output is
// bit-identical for any thread count.  Segment s covers genome offsets
// [s*R*5, (s+1)*R*5) in sorted mode, i.e. ~30x coverage of 150 bp reads.
//
// C ABI (ctypes): hbamgen_generate_file / hbamgen_generate_mem / hbamgen_free.
// CLI: gen_bam OUT.bam [--records N | --target-bytes C] [--seed S] ...

#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

extern "C" {

struct hbamgen_params {
  uint64_t n_records;        // records to emit (mapped + unmapped); 0 = use target_bytes
  uint64_t target_bytes;     // stop after this many compressed bytes (approx, segment granular)
  uint64_t seed;
  int32_t sorted;            // 1 = coordinate sorted, 0 = shuffled order
  int32_t qual_model;        // 0 = binned {2,12,23,37} + 5 % noise, 1 = uniform Q2..Q41
  int32_t block_payload;     // uncompressed bytes per full BGZF block (<= 65536)
  int32_t straddle;          // 1 = records straddle blocks (htsjdk), 0 = never (htslib)
  int32_t level;             // zlib level (htsjdk default 5)
  int32_t threads;
  int32_t segment_records;   // records per independently-compressed segment
  int32_t empty_block_every; // insert an empty BGZF block after every K blocks (0 = never)
  int32_t long_read_every;   // every K-th record gets a >64 KiB sequence (0 = never)
  int32_t odd_every;         // every K-th record gets an odd/short l_seq, 0xFF qual, etc.
  int32_t unplaced_permille; // unplaced unmapped reads at end of sorted file (default 5)
  int32_t mate_unmapped_permille;  // default 10
  int32_t write_terminator;  // append the 28-byte EOF block
  int32_t n_ref;             // reference sequences in the dictionary (<= 25 named, more synthetic)
};

void hbamgen_default_params(hbamgen_params* p);
int hbamgen_generate_mem(const hbamgen_params* p, uint8_t** out, uint64_t* out_len,
                         uint64_t* n_records_out);
int hbamgen_generate_file(const hbamgen_params* p, const char* path, uint64_t* out_len,
                          uint64_t* n_records_out);
void hbamgen_free(uint8_t* p);
// Byte range of ONE file made of `n_seg_total` main segments (target_bytes / n_records are
// ignored): segments [seg_first, seg_first + seg_count), preceded by the header blocks when
// flags & 1, followed by the unplaced-unmapped tail and the terminator when flags & 2.  The
// concatenation of consecutive ranges (header on the first, tail on the last) is the file
// hbamgen_generate_mem writes for n_records = n_seg_total * segment_records (+ the unplaced
// tail).  Requires empty_block_every == 0 (empty blocks use a file-global block counter).
int hbamgen_generate_range(const hbamgen_params* p, uint64_t n_seg_total, uint64_t seg_first,
                           uint64_t seg_count, int32_t flags, uint8_t** out, uint64_t* out_len,
                           uint64_t* n_records_out);
}

namespace {

const char* kContigNames[25] = {"chr1",  "chr2",  "chr3",  "chr4",  "chr5",  "chr6",  "chr7",
                                "chr8",  "chr9",  "chr10", "chr11", "chr12", "chr13", "chr14",
                                "chr15", "chr16", "chr17", "chr18", "chr19", "chr20", "chr21",
                                "chr22", "chrX",  "chrY",  "chrM"};
const int64_t kContigLens[25] = {248956422, 242193529, 198295559, 190214555, 181538259,
                                 170805979, 159345973, 145138636, 138394717, 133797422,
                                 135086622, 133275309, 114364328, 107043718, 101991189,
                                 90338345,  83257441,  80373285,  58617616,  64444167,
                                 46709983,  50818468,  156040895, 57227415,  16569};

struct Rng {
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed) {}
  uint64_t next() {
    uint64_t z = (s += 0x9e3779b97f4a7c15ULL);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
  }
  uint32_t below(uint32_t n) { return (uint32_t)((next() >> 32) * (uint64_t)n >> 32); }
};

uint64_t mix(uint64_t a, uint64_t b) {
  Rng r(a * 0x100000001b3ULL ^ (b + 0x632be59bd9b4e019ULL));
  r.next();
  return r.next();
}

struct Genome {
  int n_ref;
  std::vector<std::string> names;
  std::vector<int64_t> lens;
  std::vector<int64_t> cum;  // cumulative start
  int64_t total = 0;
  explicit Genome(int n) : n_ref(n) {
    for (int i = 0; i < n; ++i) {
      if (i < 25) {
        names.push_back(kContigNames[i]);
        lens.push_back(kContigLens[i]);
      } else {
        names.push_back("chrUn_" + std::to_string(i));
        lens.push_back(100000 + 1000 * i);
      }
      cum.push_back(total);
      total += lens.back();
    }
  }
  // genome offset -> (refID, pos); wraps around the genome
  void locate(int64_t g, int32_t* ref, int32_t* pos) const {
    g %= total;
    int lo = 0, hi = n_ref - 1;
    while (lo < hi) {
      int mid = (lo + hi + 1) / 2;
      if (cum[mid] <= g) lo = mid; else hi = mid - 1;
    }
    *ref = lo;
    *pos = (int32_t)(g - cum[lo]);
  }
};

void put32(std::string& s, uint32_t v) { s.append((const char*)&v, 4); }
void put16(std::string& s, uint16_t v) { s.append((const char*)&v, 2); }
void put8(std::string& s, uint8_t v) { s.push_back((char)v); }

int reg2bin(int beg, int end) {
  --end;
  if (beg >> 14 == end >> 14) return ((1 << 15) - 1) / 7 + (beg >> 14);
  if (beg >> 17 == end >> 17) return ((1 << 12) - 1) / 7 + (beg >> 17);
  if (beg >> 20 == end >> 20) return ((1 << 9) - 1) / 7 + (beg >> 20);
  if (beg >> 23 == end >> 23) return ((1 << 6) - 1) / 7 + (beg >> 23);
  if (beg >> 26 == end >> 26) return ((1 << 3) - 1) / 7 + (beg >> 26);
  return 0;
}

std::string make_header_bytes(const Genome& g, bool sorted) {
  std::string text = std::string("@HD\tVN:1.6\tSO:") + (sorted ? "coordinate" : "unsorted") + "\n";
  for (int i = 0; i < g.n_ref; ++i)
    text += "@SQ\tSN:" + g.names[i] + "\tLN:" + std::to_string(g.lens[i]) + "\n";
  text += "@RG\tID:grp1\tSM:sample1\tPL:ILLUMINA\tLB:lib1\n";
  text += "@PG\tID:gen_bam\tPN:gen_bam\tVN:1\n";
  std::string h = "BAM\1";
  put32(h, (uint32_t)text.size());
  h += text;
  put32(h, (uint32_t)g.n_ref);
  for (int i = 0; i < g.n_ref; ++i) {
    put32(h, (uint32_t)(g.names[i].size() + 1));
    h += g.names[i];
    put8(h, 0);
    put32(h, (uint32_t)g.lens[i]);
  }
  return h;
}

static const char kBases[] = "ACGT";

struct RecordSpec {
  int32_t ref, pos, next_ref, next_pos, tlen;
  uint16_t flag;
  uint8_t mapq;
  bool unmapped_nocigar;
};

// Appends one BAM record (block_size-prefixed) to out.
void emit_record(std::string& out, Rng& r, const hbamgen_params& P, uint64_t rec_index,
                 const RecordSpec& rs) {
  int l_seq = 150;
  bool odd = P.odd_every > 0 && rec_index % (uint64_t)P.odd_every == (uint64_t)(P.odd_every - 1);
  bool longread =
      P.long_read_every > 0 && rec_index % (uint64_t)P.long_read_every == (uint64_t)(P.long_read_every - 1);
  int odd_kind = odd ? (int)(r.below(4)) : -1;
  if (odd) {
    if (odd_kind == 0) l_seq = 1 + (int)r.below(300);       // ragged length (often odd)
    else if (odd_kind == 1) l_seq = 0;                      // SEQ '*'
    else if (odd_kind == 2) l_seq = 151;                    // odd length
    else l_seq = 37;                                        // short, 0xFF qual below
  }
  if (longread) l_seq = 70000 + (int)r.below(20000);

  // read name
  char name[64];
  int nl = snprintf(name, sizeof name, "A00%03u:%u:H%05uDSX:%u:%u:%u:%u",
                    (unsigned)(rec_index >> 20) % 1000, (unsigned)(rec_index >> 14) % 97,
                    (unsigned)(rec_index % 99991), (unsigned)(rec_index & 3) + 1,
                    1101 + (unsigned)r.below(2000), (unsigned)r.below(32000),
                    (unsigned)(rec_index >> 1) % 40000);
  // CIGAR
  std::vector<uint32_t> cig;
  if (!rs.unmapped_nocigar && l_seq > 0) {
    uint32_t u = r.below(100);
    if (u < 90 || l_seq < 20 || longread) {
      cig.push_back((uint32_t)l_seq << 4 | 0);  // M
    } else if (u < 95) {
      int clip = 1 + (int)r.below(15);
      if (r.below(2)) {
        cig.push_back((uint32_t)clip << 4 | 4);
        cig.push_back((uint32_t)(l_seq - clip) << 4 | 0);
      } else {
        cig.push_back((uint32_t)(l_seq - clip) << 4 | 0);
        cig.push_back((uint32_t)clip << 4 | 4);
      }
    } else {
      int ilen = 1 + (int)r.below(3);
      int a = 20 + (int)r.below((uint32_t)std::max(1, l_seq - 40 - ilen));
      if (r.below(2)) {  // insertion consumes query
        cig.push_back((uint32_t)a << 4 | 0);
        cig.push_back((uint32_t)ilen << 4 | 1);
        cig.push_back((uint32_t)(l_seq - a - ilen) << 4 | 0);
      } else {           // deletion does not
        cig.push_back((uint32_t)a << 4 | 0);
        cig.push_back((uint32_t)ilen << 4 | 2);
        cig.push_back((uint32_t)(l_seq - a) << 4 | 0);
      }
    }
  }
  int ref_span = 0;
  for (uint32_t c : cig) {
    int op = c & 15;
    if (op == 0 || op == 2 || op == 3 || op == 7 || op == 8) ref_span += (int)(c >> 4);
  }
  int bin = rs.pos >= 0 ? reg2bin(rs.pos, rs.pos + std::max(1, ref_span)) : 4680;
  if (rs.pos < 0) bin = 4680;

  std::string var;
  var.append(name, (size_t)nl);
  put8(var, 0);
  for (uint32_t c : cig) put32(var, c);
  // SEQ
  for (int i = 0; i < l_seq; i += 2) {
    auto code = [&](void) -> uint8_t {
      uint32_t b = r.below(1000);
      if (b == 0) return 15;  // N
      static const uint8_t acgt[4] = {1, 2, 4, 8};
      return acgt[b & 3];
    };
    uint8_t hi = code(), lo = (i + 1 < l_seq) ? code() : 0;
    put8(var, (uint8_t)(hi << 4 | lo));
  }
  // QUAL
  if (odd_kind == 3) {
    for (int i = 0; i < l_seq; ++i) put8(var, 0xff);
  } else if (P.qual_model == 1) {
    for (int i = 0; i < l_seq; ++i) put8(var, (uint8_t)(2 + r.below(40)));
  } else {
    static const uint8_t bins[4] = {2, 12, 23, 37};
    for (int i = 0; i < l_seq; ++i) {
      uint32_t u = r.below(100);
      uint8_t q;
      if (u < 5) q = (uint8_t)(2 + r.below(40));
      else if (u < 75) q = 37;
      else if (u < 90) q = 23;
      else if (u < 97) q = 12;
      else q = 2;
      (void)bins;
      put8(var, q);
    }
  }
  // AUX
  if (!rs.unmapped_nocigar) {
    int nm = (int)r.below(6);
    var += "NMC"; put8(var, (uint8_t)nm);
    char md[32];
    int mdl;
    if (nm == 0) mdl = snprintf(md, sizeof md, "%d", std::max(l_seq, 0));
    else mdl = snprintf(md, sizeof md, "%d%c%d", l_seq / 2, kBases[r.below(4)],
                        std::max(0, l_seq - l_seq / 2 - 1));
    var += "MDZ"; var.append(md, (size_t)mdl); put8(var, 0);
    var += "ASC"; put8(var, (uint8_t)(l_seq > 0 ? std::min(255, l_seq - 5 * nm) : 0));
    var += "XSC"; put8(var, (uint8_t)r.below(120));
  }
  var += "RGZgrp1"; put8(var, 0);
  if (!rs.unmapped_nocigar) { var += "MCZ150M"; put8(var, 0); }

  uint32_t block_size = 32 + (uint32_t)var.size();
  put32(out, block_size);
  put32(out, (uint32_t)rs.ref);
  put32(out, (uint32_t)rs.pos);
  put8(out, (uint8_t)(nl + 1));
  put8(out, rs.mapq);
  put16(out, (uint16_t)bin);
  put16(out, (uint16_t)cig.size());
  put16(out, rs.flag);
  put32(out, (uint32_t)l_seq);
  put32(out, (uint32_t)rs.next_ref);
  put32(out, (uint32_t)rs.next_pos);
  put32(out, (uint32_t)rs.tlen);
  out += var;
}

// Uncompressed bytes of segment `seg` (records [first, first+count)).
// `unplaced` = this segment holds only unplaced unmapped reads.
std::string make_segment(const hbamgen_params& P, const Genome& g, uint64_t seg, uint64_t first,
                         uint64_t count, bool unplaced, std::vector<uint32_t>* rec_sizes) {
  std::string out;
  out.reserve(count * 360);
  Rng r(mix(P.seed, seg));
  const int64_t seg_base = (int64_t)(first * 5);
  for (uint64_t i = 0; i < count; ++i) {
    uint64_t ri = first + i;
    RecordSpec rs{};
    size_t before = out.size();
    if (unplaced) {
      rs = RecordSpec{-1, -1, -1, -1, 0, (uint16_t)((i & 1) ? 141 : 77), 0, true};
    } else {
      int64_t goff;
      if (P.sorted) goff = seg_base + (int64_t)i * 5 + (int64_t)r.below(5);
      else goff = (int64_t)(r.next() % (uint64_t)g.total);
      int32_t ref, pos;
      g.locate(goff, &ref, &pos);
      int insert = 300 + (int)r.below(101);
      uint32_t u = r.below(1000);
      bool mate_unmapped = u < (uint32_t)P.mate_unmapped_permille;
      if (mate_unmapped) {
        // mapped read whose mate is unmapped (73/137), or the placed-unmapped mate (133/69)
        uint32_t k = r.below(4);
        static const uint16_t fl[4] = {73, 137, 133, 69};
        bool self_unmapped = (k >= 2);
        rs = RecordSpec{ref, pos, ref, pos, 0, fl[k], (uint8_t)(self_unmapped ? 0 : 60), self_unmapped};
      } else {
        static const uint16_t fl[4] = {99, 147, 83, 163};
        uint16_t f = fl[r.below(4)];
        bool mate_fwd = (f == 147 || f == 83);
        int32_t npos = mate_fwd ? pos - insert + 150 : pos + insert - 150;
        if (npos < 0) npos = 0;
        int32_t tlen = mate_fwd ? -insert : insert;
        uint8_t mapq = r.below(10) == 0 ? (uint8_t)r.below(60) : 60;
        rs = RecordSpec{ref, pos, ref, npos, tlen, f, mapq, false};
      }
    }
    emit_record(out, r, P, ri, rs);
    if (rec_sizes) rec_sizes->push_back((uint32_t)(out.size() - before));
  }
  return out;
}

struct Compressor {
  z_stream zs;
  z_stream zs0;
  explicit Compressor(int level) {
    memset(&zs, 0, sizeof zs);
    memset(&zs0, 0, sizeof zs0);
    deflateInit2(&zs, level, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY);
    deflateInit2(&zs0, 0, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY);
  }
  ~Compressor() {
    deflateEnd(&zs);
    deflateEnd(&zs0);
  }
  // Appends one BGZF block holding `n` bytes of `src`.
  void block(std::string& out, const uint8_t* src, size_t n) {
    uint8_t buf[65536];
    const size_t cap = 65536 - 26;
    z_stream* z = &zs;
    deflateReset(z);
    z->next_in = (Bytef*)src;
    z->avail_in = (uInt)n;
    z->next_out = buf + 18;
    z->avail_out = (uInt)cap;
    int rc = deflate(z, Z_FINISH);
    if (rc != Z_STREAM_END) {  // does not fit: store, like htsjdk's no-compression fallback
      z = &zs0;
      deflateReset(z);
      z->next_in = (Bytef*)src;
      z->avail_in = (uInt)n;
      z->next_out = buf + 18;
      z->avail_out = (uInt)cap;
      rc = deflate(z, Z_FINISH);
      if (rc != Z_STREAM_END) { fprintf(stderr, "gen_bam: block does not fit\n"); abort(); }
    }
    size_t clen = cap - z->avail_out;
    size_t total = clen + 26;
    static const uint8_t hdr[16] = {0x1f, 0x8b, 8, 4, 0, 0, 0, 0, 0, 0xff, 6, 0, 'B', 'C', 2, 0};
    memcpy(buf, hdr, 16);
    uint16_t bsize = (uint16_t)(total - 1);
    memcpy(buf + 16, &bsize, 2);
    uint32_t crc = (uint32_t)crc32(0L, src, (uInt)n);
    uint32_t isz = (uint32_t)n;
    memcpy(buf + 18 + clen, &crc, 4);
    memcpy(buf + 22 + clen, &isz, 4);
    out.append((const char*)buf, total);
  }
};

const uint8_t kEof[28] = {0x1f, 0x8b, 8, 4, 0, 0, 0, 0, 0, 0xff, 6, 0, 0x42, 0x43,
                          2,    0,    0x1b, 0, 3, 0, 0, 0, 0, 0, 0, 0, 0, 0};

// Compresses a segment's uncompressed bytes into BGZF blocks.
std::string compress_segment(const hbamgen_params& P, const std::string& u,
                             const std::vector<uint32_t>& rec_sizes, Compressor& c,
                             uint64_t* blocks_emitted, uint64_t block_counter_base) {
  std::string out;
  out.reserve(u.size() / 2 + 1024);
  const size_t B = (size_t)P.block_payload;
  uint64_t nb = 0;
  auto maybe_empty = [&]() {
    ++nb;
    if (P.empty_block_every > 0 && (block_counter_base + nb) % (uint64_t)P.empty_block_every == 0)
      out.append((const char*)kEof, 28);
  };
  if (P.straddle) {
    for (size_t off = 0; off < u.size(); off += B) {
      size_t n = std::min(B, u.size() - off);
      c.block(out, (const uint8_t*)u.data() + off, n);
      maybe_empty();
    }
  } else {
    size_t start = 0, cur = 0;
    for (uint32_t rs : rec_sizes) {
      if (cur + rs - start > B && cur > start) {
        c.block(out, (const uint8_t*)u.data() + start, cur - start);
        maybe_empty();
        start = cur;
      }
      cur += rs;
      while (cur - start > B) {  // a single record larger than a block: it must straddle
        c.block(out, (const uint8_t*)u.data() + start, B);
        maybe_empty();
        start += B;
      }
    }
    if (cur > start) {
      c.block(out, (const uint8_t*)u.data() + start, cur - start);
      maybe_empty();
    }
  }
  *blocks_emitted = nb;
  return out;
}

template <class Sink>
int generate(const hbamgen_params& P0, Sink&& sink, uint64_t* n_records_out) {
  hbamgen_params P = P0;
  if (P.block_payload <= 0 || P.block_payload > 65536) P.block_payload = 65280;
  if (P.segment_records <= 0) P.segment_records = 65536;
  if (P.threads <= 0) P.threads = (int)std::max(1u, std::thread::hardware_concurrency());
  if (P.n_ref <= 0) P.n_ref = 25;
  Genome g(P.n_ref);

  // header block(s): flushed on their own, like samtools / htsjdk writeHeader + flush
  {
    Compressor c(P.level);
    std::string h = make_header_bytes(g, P.sorted != 0);
    std::string out;
    for (size_t off = 0; off < h.size(); off += (size_t)P.block_payload)
      c.block(out, (const uint8_t*)h.data() + off,
              std::min((size_t)P.block_payload, h.size() - off));
    sink(out);
  }

  uint64_t total_records = 0;
  uint64_t comp_bytes = 0;
  const uint64_t R = (uint64_t)P.segment_records;
  uint64_t main_records;  // mapped (or shuffled) records
  uint64_t unplaced_records;
  bool by_target = (P.n_records == 0);
  if (!by_target) {
    unplaced_records = P.sorted ? P.n_records * (uint64_t)P.unplaced_permille / 1000 : 0;
    main_records = P.n_records - unplaced_records;
  } else {
    main_records = UINT64_MAX;
    unplaced_records = 0;
  }

  uint64_t seg = 0;
  uint64_t block_base = 0;
  const uint64_t target_main =
      by_target ? P.target_bytes - P.target_bytes * (uint64_t)P.unplaced_permille / 1000 : 0;
  bool done = false;
  while (!done) {
    // one wave of segments in parallel
    int T = P.threads;
    std::vector<std::string> outs((size_t)T);
    std::vector<uint64_t> counts((size_t)T, 0), nblk((size_t)T, 0);
    std::vector<std::thread> th;
    uint64_t wave_first = total_records;
    int nseg = 0;
    for (int t = 0; t < T; ++t) {
      uint64_t first = wave_first + (uint64_t)t * R;
      if (!by_target && first >= main_records) break;
      counts[(size_t)t] = by_target ? R : std::min(R, main_records - first);
      ++nseg;
    }
    if (nseg == 0) break;
    for (int t = 0; t < nseg; ++t) {
      th.emplace_back([&, t]() {
        Compressor c(P.level);
        std::vector<uint32_t> sizes;
        uint64_t first = wave_first + (uint64_t)t * R;
        std::string u = make_segment(P, g, seg + (uint64_t)t, first, counts[(size_t)t], false, &sizes);
        outs[(size_t)t] = compress_segment(P, u, sizes, c, &nblk[(size_t)t], 0);
      });
    }
    for (auto& x : th) x.join();
    for (int t = 0; t < nseg; ++t) {
      // empty-block insertion uses a global block counter: recompute deterministically
      if (P.empty_block_every > 0) {
        Compressor c(P.level);
        std::vector<uint32_t> sizes;
        uint64_t first = wave_first + (uint64_t)t * R;
        std::string u = make_segment(P, g, seg + (uint64_t)t, first, counts[(size_t)t], false, &sizes);
        outs[(size_t)t] = compress_segment(P, u, sizes, c, &nblk[(size_t)t], block_base);
      }
      block_base += nblk[(size_t)t];
      sink(outs[(size_t)t]);
      comp_bytes += outs[(size_t)t].size();
      total_records += counts[(size_t)t];
      if (by_target && comp_bytes >= target_main) { done = true; seg += (uint64_t)t + 1; break; }
    }
    if (!done) seg += (uint64_t)nseg;
    if (!by_target && total_records >= main_records) done = true;
  }
  if (by_target && P.sorted) unplaced_records = total_records * (uint64_t)P.unplaced_permille / 1000;
  // unplaced unmapped reads at the end (sorted files only)
  for (uint64_t first = 0; first < unplaced_records; first += R) {
    uint64_t cnt = std::min(R, unplaced_records - first);
    Compressor c(P.level);
    std::vector<uint32_t> sizes;
    std::string u = make_segment(P, g, 0x7fff0000ULL + first / R, total_records, cnt, true, &sizes);
    uint64_t nb = 0;
    std::string o = compress_segment(P, u, sizes, c, &nb, block_base);
    block_base += nb;
    sink(o);
    total_records += cnt;
  }
  if (P.write_terminator) sink(std::string((const char*)kEof, 28));
  if (n_records_out) *n_records_out = total_records;
  return 0;
}

}  // namespace

extern "C" {

void hbamgen_default_params(hbamgen_params* p) {
  memset(p, 0, sizeof *p);
  p->n_records = 20000;
  p->seed = 1;
  p->sorted = 1;
  p->qual_model = 0;
  p->block_payload = 65280;
  p->straddle = 1;
  p->level = 5;
  p->threads = 0;
  p->segment_records = 65536;
  p->unplaced_permille = 5;
  p->mate_unmapped_permille = 10;
  p->write_terminator = 1;
  p->n_ref = 25;
}

int hbamgen_generate_mem(const hbamgen_params* p, uint8_t** out, uint64_t* out_len,
                         uint64_t* n_records_out) {
  std::string* acc = new std::string();
  generate(*p, [&](const std::string& s) { acc->append(s); }, n_records_out);
  uint8_t* buf = (uint8_t*)malloc(acc->size() ? acc->size() : 1);
  if (!buf) { delete acc; return -1; }
  memcpy(buf, acc->data(), acc->size());
  *out = buf;
  *out_len = acc->size();
  delete acc;
  return 0;
}

int hbamgen_generate_file(const hbamgen_params* p, const char* path, uint64_t* out_len,
                          uint64_t* n_records_out) {
  FILE* f = fopen(path, "wb");
  if (!f) return -1;
  uint64_t n = 0;
  generate(*p, [&](const std::string& s) { fwrite(s.data(), 1, s.size(), f); n += s.size(); },
           n_records_out);
  fclose(f);
  if (out_len) *out_len = n;
  return 0;
}

void hbamgen_free(uint8_t* p) { free(p); }

int hbamgen_generate_range(const hbamgen_params* p0, uint64_t n_seg_total, uint64_t seg_first,
                           uint64_t seg_count, int32_t flags, uint8_t** out, uint64_t* out_len,
                           uint64_t* n_records_out) {
  hbamgen_params P = *p0;
  if (P.empty_block_every != 0 || seg_first + seg_count > n_seg_total) return -1;
  if (P.block_payload <= 0 || P.block_payload > 65536) P.block_payload = 65280;
  if (P.segment_records <= 0) P.segment_records = 65536;
  if (P.threads <= 0) P.threads = (int)std::max(1u, std::thread::hardware_concurrency());
  if (P.n_ref <= 0) P.n_ref = 25;
  Genome g(P.n_ref);
  const uint64_t R = (uint64_t)P.segment_records;
  std::string acc;
  uint64_t nrec = 0;
  if (flags & 1) {
    Compressor c(P.level);
    std::string h = make_header_bytes(g, P.sorted != 0);
    for (size_t off = 0; off < h.size(); off += (size_t)P.block_payload)
      c.block(acc, (const uint8_t*)h.data() + off, std::min((size_t)P.block_payload, h.size() - off));
  }
  std::vector<std::string> outs((size_t)seg_count);
  std::atomic<uint64_t> next{0};
  std::vector<std::thread> th;
  for (int t = 0; t < P.threads; ++t)
    th.emplace_back([&]() {
      Compressor c(P.level);
      for (uint64_t k; (k = next.fetch_add(1)) < seg_count;) {
        std::vector<uint32_t> sizes;
        const uint64_t seg = seg_first + k;
        std::string u = make_segment(P, g, seg, seg * R, R, false, &sizes);
        uint64_t nb = 0;
        outs[(size_t)k] = compress_segment(P, u, sizes, c, &nb, 0);
      }
    });
  for (auto& x : th) x.join();
  for (auto& o : outs) acc += o;
  nrec += seg_count * R;
  if (flags & 2) {
    const uint64_t main_records = n_seg_total * R;
    const uint64_t unplaced = P.sorted ? main_records * (uint64_t)P.unplaced_permille / 1000 : 0;
    for (uint64_t first = 0; first < unplaced; first += R) {
      const uint64_t cnt = std::min(R, unplaced - first);
      Compressor c(P.level);
      std::vector<uint32_t> sizes;
      std::string u = make_segment(P, g, 0x7fff0000ULL + first / R, main_records, cnt, true, &sizes);
      uint64_t nb = 0;
      acc += compress_segment(P, u, sizes, c, &nb, 0);
      nrec += cnt;
    }
    if (P.write_terminator) acc.append((const char*)kEof, 28);
  }
  uint8_t* buf = (uint8_t*)malloc(acc.size() ? acc.size() : 1);
  if (!buf) return -1;
  memcpy(buf, acc.data(), acc.size());
  *out = buf;
  *out_len = acc.size();
  if (n_records_out) *n_records_out = nrec;
  return 0;
}

}  // extern "C"

#ifdef HBAMGEN_MAIN
int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr,
            "usage: gen_bam OUT.bam [--records N] [--target-bytes C] [--seed S] [--unsorted]\n"
            "       [--uniform-qual] [--htslib] [--payload B] [--level L] [--threads T]\n"
            "       [--segment R] [--empty-every K] [--long-every K] [--odd-every K]\n"
            "       [--no-terminator] [--n-ref N]\n");
    return 2;
  }
  hbamgen_params p;
  hbamgen_default_params(&p);
  for (int i = 2; i < argc; ++i) {
    std::string a = argv[i];
    auto nx = [&]() { return (i + 1 < argc) ? strtoull(argv[++i], nullptr, 0) : 0ULL; };
    if (a == "--records") p.n_records = nx();
    else if (a == "--target-bytes") { p.target_bytes = nx(); p.n_records = 0; }
    else if (a == "--seed") p.seed = nx();
    else if (a == "--unsorted") p.sorted = 0;
    else if (a == "--uniform-qual") p.qual_model = 1;
    else if (a == "--htslib") p.straddle = 0;
    else if (a == "--payload") p.block_payload = (int)nx();
    else if (a == "--level") p.level = (int)nx();
    else if (a == "--threads") p.threads = (int)nx();
    else if (a == "--segment") p.segment_records = (int)nx();
    else if (a == "--empty-every") p.empty_block_every = (int)nx();
    else if (a == "--long-every") p.long_read_every = (int)nx();
    else if (a == "--odd-every") p.odd_every = (int)nx();
    else if (a == "--no-terminator") p.write_terminator = 0;
    else if (a == "--n-ref") p.n_ref = (int)nx();
    else { fprintf(stderr, "unknown option %s\n", a.c_str()); return 2; }
  }
  uint64_t len = 0, nrec = 0;
  if (hbamgen_generate_file(&p, argv[1], &len, &nrec) != 0) { perror(argv[1]); return 1; }
  printf("%s: %llu bytes, %llu records\n", argv[1], (unsigned long long)len,
         (unsigned long long)nrec);
  return 0;
}
#endif
