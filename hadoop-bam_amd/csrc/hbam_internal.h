// hbam_internal.h — definitions shared by the kernels and the host runtime (not public ABI).
#pragma once
#include <stdint.h>

#include "../../include/hbam.h"

namespace hbam {

constexpr uint32_t SCAN_CHUNK = 65536;  // bytes per scan workgroup (multiple of 256*16)
constexpr uint32_t SCAN_CAP = 64;       // candidate slots per chunk
constexpr uint32_t INFLATE_WG = 64;     // lanes (= blocks) per inflate workgroup
constexpr uint32_t LENS_SLOT = 352;     // per-block global scratch for code lengths
constexpr uint32_t BITMAP_WORDS = 2048;  // per-block match-start bitmap (65536 bits)
constexpr uint32_t WALK_CAP = 1880;     // >= 65536/35 record starts per block (BAM >= 36 B, BCF >= 35 B)
constexpr uint32_t SCAN_WG = 256;
constexpr uint32_t POOLS_MAX_WG = 8192;    // k_decode_pools grid cap (grid-stride over records)
constexpr uint32_t GATHER_MAX_WG = 65536;  // k_gather_records grid cap (grid-stride over records)
constexpr uint64_t UBUF_SLACK = 8192;  // k_resolve reads whole 2 KiB stretches past a block end
constexpr uint32_t SCAN_TILE = 4096;
constexpr uint64_t NO_ENTRY = ~0ULL;
constexpr uint64_t CHAIN_STOP = ~0ULL - 1;

// per-record status (decode) — values < 0 are HBAM_E* codes
enum : int32_t {
  ST_OK = 0,
  ST_NULL = 1,  // decode() returned null: clean end of the split
  ST_VEND = 2,  // getFilePointer() >= vEnd: clean end of the split
};

struct BlockRec {
  uint64_t coff;   // offset of the block in the device buffer
  uint32_t clen;   // BSIZE + 1
  uint32_t isize;  // ISIZE footer
  uint32_t crc;    // CRC32 footer
  uint32_t pad;
};

// Device column set (struct-of-arrays) passed by value to kernels.
struct DevColumns {
  int32_t* status;
  int32_t* block_size;
  int32_t* ref_id;
  int32_t* pos;
  uint8_t* l_read_name;
  uint8_t* mapq;
  uint16_t* bin;
  uint16_t* n_cigar;
  uint16_t* flag;
  int32_t* l_seq;
  int32_t* next_ref_id;
  int32_t* next_pos;
  int32_t* tlen;
  int64_t* key;
  uint8_t* layout_ok;
  uint32_t* name_len;
  uint32_t* cigar_n;
  uint32_t* seq_len;
  uint32_t* aux_len;
  uint64_t* name_off;
  uint64_t* cigar_off;
  uint64_t* seq_off;
  uint64_t* aux_off;
  uint8_t* names;
  uint32_t* cigars;
  uint8_t* seq;
  uint8_t* qual;
  uint8_t* aux;
};

}  // namespace hbam
