// Byte -> code table shared by the encoders (encode.hip) and the fused whitelist ingest
// (lines.hip).  Reference maps: TwoBit encodings.py:53-69, ThreeBit encodings.py:139-149.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr uint8_t F_AMBIG = 0x40, F_INVALID = 0x80;

// Pointers typed as LDS (address space 3): reads through them are ds_read.  A generic pointer
// that may point at LDS or at global memory compiles to flat loads, and the compiler waits
// vmcnt(0) AND lgkmcnt(0) after every flat load -- draining the tile prefetch and every
// outstanding store of the workgroup's loop each time (the ingest kernels' tile loops).
typedef __attribute__((address_space(3))) const uint32_t lds_u32;
typedef __attribute__((address_space(3))) const uint8_t lds_u8;
typedef __attribute__((address_space(3))) const uint16_t lds_u16;
template <class T>
__device__ __forceinline__ lds_u32* as_lds32(T* p) {
  return (lds_u32*)(p);
}
template <class T>
__device__ __forceinline__ lds_u8* as_lds8(T* p) {
  return (lds_u8*)(p);
}
template <class T>
__device__ __forceinline__ lds_u16* as_lds16(T* p) {
  return (lds_u16*)(p);
}

// LUT entry: low 3 bits = code, 0x40 = IUPAC ambiguous (TwoBit), 0x80 = invalid (TwoBit)
__host__ __device__ inline uint8_t lut_entry(int kind, int c) {
  if (kind == 2) {
    switch (c) {
      case 'A': case 'a': return 0;
      case 'C': case 'c': return 1;
      case 'T': case 't': return 2;
      case 'G': case 'g': return 3;
      case 'M': case 'R': case 'W': case 'S': case 'Y': case 'K': case 'V': case 'H': case 'D':
      case 'B': case 'N': case 'm': case 'r': case 'w': case 's': case 'y': case 'k': case 'v':
      case 'h': case 'd': case 'b': case 'n':
        return F_AMBIG;
      default: return F_INVALID;
    }
  }
  switch (c) {
    case 'C': case 'c': return 1;
    case 'A': case 'a': return 2;
    case 'G': case 'g': return 3;
    case 'T': case 't': return 4;
    default: return 6;  // N/n and every other byte
  }
}


// Read byte p of a record either through aligned dwords or bytes.
struct RecordReader {
  const uint8_t* rec;
  bool dw;
  uint32_t cache;
  int cache_k;
  __device__ __forceinline__ uint32_t byte(int p) {
    if (dw) {
      const int k = p >> 2;
      if (k != cache_k) {
        cache = *reinterpret_cast<const uint32_t*>(rec + 4 * k);
        cache_k = k;
      }
      return (cache >> (8 * (p & 3))) & 0xFFu;
    }
    return rec[p];
  }
};

// One record of L bytes through the byte LUT into `words` limbs of out; returns the GC
// count (capped at 255 by the callers) and the ambiguous / invalid flags (bits 0 / 1).
__device__ __forceinline__ void encode_record(const uint8_t* lut, int bits, RecordReader& rd, int L, int words,
                                              uint64_t* out, uint32_t& g, uint32_t& flag_bits) {
  uint32_t fl = 0;
  g = 0;
  if (words == 1) {
    uint64_t code = 0;
    for (int p = 0; p < L; ++p) {
      const uint32_t e = lut[rd.byte(p)];
      code = (code << bits) | (e & 7u);
      fl |= e;
    }
    out[0] = code;
    const uint64_t m = bits == 2 ? 0x5555555555555555ull : 0x9249249249249249ull;
    g = __popcll(code & m);
  } else {
    // LSB-first over positions so limbs complete in order; a triplet may straddle limbs.
    uint64_t cur = 0, nxt = 0;
    int wcur = 0;
    for (int p = L - 1; p >= 0; --p) {
      const uint32_t e = lut[rd.byte(p)];
      fl |= e;
      const uint64_t v = e & 7u;
      g += (uint32_t)(v & 1u);
      const int64_t pos = (int64_t)bits * (L - 1 - p);
      const int w = (int)(pos >> 6), off = (int)(pos & 63);
      while (w > wcur) {
        out[wcur++] = cur;
        cur = nxt;
        nxt = 0;
      }
      cur |= v << off;
      if (off + bits > 64) nxt |= v >> (64 - off);
    }
    out[wcur++] = cur;
    if (wcur < words) out[wcur++] = nxt;
    while (wcur < words) out[wcur++] = 0;
  }
  flag_bits = ((fl & F_AMBIG) ? 1u : 0u) | ((fl & F_INVALID) ? 2u : 0u);
}

}  // namespace
