/*
 * sctools_hip.h — C ABI of libsctools_hip.so, the MI355X (gfx950) barcode hot path.
 *
 * The reference (dpeerlab/sctools) is pure Python and has no FFI of its own; each
 * entry point below replaces the Python function cited next to it, and the Python
 * drop-in (sctools_amd.encodings / sctools_amd.barcode) binds them with ctypes
 * (INTEGRATION.md shows the binding).  Conventions:
 *   - every function returns an int status: SCT_OK (0) or a negative SCT_E_* code;
 *     sct_last_error() returns a thread-local message for the last failure;
 *   - "device" functions take device pointers and a hipStream_t passed as void*
 *     (NULL = the default stream) and are asynchronous on that stream;
 *   - "_host" functions take host pointers, run on the current device and return
 *     only when results are back in host memory;
 *   - codes wider than 64 bits are `words` little-endian uint64 limbs per record
 *     (limb 0 holds bits 0..63 of the Python int);
 *   - no function retains a caller pointer after it returns (plans own their
 *     device buffers and hold no host pointers).
 */
#ifndef SCTOOLS_HIP_H
#define SCTOOLS_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SCT_OK 0
#define SCT_E_INVALID (-1)   /* bad argument (maps to ValueError)             */
#define SCT_E_HIP (-2)       /* HIP runtime failure / no device (RuntimeError) */
#define SCT_E_NOMEM (-3)     /* device allocation failed (MemoryError)         */
#define SCT_E_RANGE (-4)     /* value outside what the kernel supports         */

/* ---------------------------------------------------------------- library */
int sct_version(void);                 /* ABI version, currently 1 */
const char* sct_last_error(void);      /* thread-local, never NULL */
int sct_device_count(int* count);      /* HIP devices visible to this process */
int sct_set_device(int device);        /* select the device for later calls (hipSetDevice) */

/* Launch-shape knobs.  None changes a result: they cut work into other chunk / grid sizes
 * or pick between index layouts that give identical outputs, so tests can put seams inside
 * small problems and benchmarks can sweep.  Process-global; the library reads no environment
 * variable.  value < 0 restores the default.  Read when a plan is created (scalar: per call). */
#define SCT_TUNE_SPECTRAL_CHUNK 1       /* slices per seed/tile pass (default 262144, the whole space; 65536 for SCT_ALLPAIRS_NO_CACHE plans) */
#define SCT_TUNE_SPECTRAL_MIN_N 2       /* AUTO takes SPECTRAL from this many 16-base codes (325000) */
#define SCT_TUNE_ALLPAIRS_GRAB 3        /* pair kernel: work items per queue pull */
#define SCT_TUNE_ALLPAIRS_FLUSH_ITEMS 4 /* pair kernel: flush lane counters every k items */
#define SCT_TUNE_ALLPAIRS_GRID 5        /* pair kernel: persistent grid size */
#define SCT_TUNE_NEAREST_SCHEME 6       /* 0 auto, 1 open addressing, 2 CSR buckets, 3 half keys */
#define SCT_TUNE_NEAREST_LOAD 7         /* open addressing: table slots per whitelist code */
#define SCT_TUNE_SCALAR_SERVER 8        /* 0: every scalar call is a kernel launch (default 1) */
#define SCT_TUNE_SCALAR_IDLE_MS 9       /* the scalar server exits after this idle time (5) */
#define SCT_TUNE_SPECTRAL_COLUMNS 10   /* SPECTRAL column width: 0 auto, 14, or 16 (when int8 fits) */
#define SCT_TUNE_PLAN_CACHE 11          /* 0: every all-pairs plan allocates its own buffers (default 1) */
#define SCT_TUNE_ENCODE_GRID 12         /* tiled encoder grid: 1 one workgroup per tile (default), 0 resident workgroups */
#define SCT_TUNE_INGEST_TILES 13        /* whitelist / FASTQ extraction: tiles per workgroup (0: one range per
                                           resident slot, the whitelist's default; FASTQ default 8) */
#define SCT_TUNE_FASTQ_ONEPASS 14       /* retired in round 5 (the one-pass FASTQ forms lost their A/B and were
                                           removed); accepted and ignored, so the key numbers stay stable */
#define SCT_TUNE_INGEST_DIRECT 15       /* whitelist ingest: up to this many 16 KiB tiles (4096) the encode pass
                                           sums the per-tile counts itself, no reduction launch */
#define SCT_TUNE_INGEST_SPEC 16         /* whitelist ingest: 1 tries 16-base lines in one read first (default), 0 never */
#define SCT_TUNE_NKEYS 17
int sct_tune_set(int key, int64_t value);
int sct_tune_get(int key, int64_t* value);  /* -1 when unset */

/* ---------------------------------------------------------------- encoders
 * kind = 2 (TwoBit) or 3 (ThreeBit).
 * Replaces TwoBit.encode  (src/sctools/encodings.py:75-88, map :53-69) and
 *          ThreeBit.encode (src/sctools/encodings.py:155-167, map :139-149).
 * n records of L bytes, record r starting at seqs + r*stride (stride >= L).
 * codes : n*words uint64, words = ceil(kind*L/64) (at least 1); MSB-first packing
 *         exactly as the reference's `encoded <<= bits; encoded += map[byte]`.
 * gc    : nullable; n uint8 = GC count of the record (requires L <= 255).
 *         TwoBit: C/c/G/g bytes (the ambiguous positions are counted after the
 *         host fills them, see flags). ThreeBit: popcount of bit 0 of each triplet
 *         (encodings.py:182-192), i.e. C/c/G/g bytes.
 * flags : nullable (TwoBit); n uint8, bit0 = an IUPAC-ambiguous byte was seen
 *         (encoded as 0, to be drawn by the caller's random.randint(0,3) in order,
 *         encodings.py:69), bit1 = an invalid byte was seen (reference raises
 *         KeyError, encodings.py:68).  ThreeBit never flags (any byte -> N=6).
 */
int sct_encode(int kind, const uint8_t* seqs, int64_t n, int64_t stride, int L,
               uint64_t* codes, uint8_t* gc, uint8_t* flags, void* stream);
int sct_encode_host(int kind, const uint8_t* seqs, int64_t n, int64_t stride, int L,
                    uint64_t* codes, uint8_t* gc, uint8_t* flags);

/* Host-resident stream of n records (stride L, one limb: L <= 32 TwoBit / 21 ThreeBit):
 * chunks of `chunk` records (<= 0: 16M) pipeline H2D / encode / D2H over 3 streams.  Buffers
 * already page-locked (sct_host_pinned) are copied by DMA in place; pageable ones go through
 * the library's own pinned stage in chunks of <= 2M records (the library never registers
 * caller memory).  gc and flags are required.  Returns when all outputs are in host memory.
 * Replaces the per-record loop of encodings.py:60-71 / 140-147 for a batch of records. */
int sct_encode_stream_host(int kind, const uint8_t* seqs, int64_t n, int L, uint64_t* codes,
                           uint8_t* gc, uint8_t* flags, int64_t chunk);

/* *pinned = 1 when all of [p, p + bytes) lies in one page-locked host allocation the HIP
 * runtime knows (hipHostMalloc, torch pin_memory, hipHostRegister): the host-stream entry
 * points then DMA to / from it in place; 0 otherwise (pageable memory, or a range that
 * runs past its allocation). */
int sct_host_pinned(const void* p, int64_t bytes, int* pinned);

/* Page-locked host blocks (hipHostMalloc) for the Python layer's pinned array pool: the host
 * stream paths (FASTQ pieces read from files, their extracted rows, stream-encoded codes,
 * nearest results) then cross PCIe by DMA in place, and a block handed back to the pool is
 * reused without new page faults.  sct_host_free(NULL) is a no-op. */
int sct_host_alloc(int64_t bytes, void** ptr);
int sct_host_free(void* ptr);

/* Variable-length records (device): record r = starts[r] .. starts[r] + lens[r] of buf,
 * encoded as encodings.py:75-88 / :155-167 do into `words` limbs (words >= ceil(kind*len/64)
 * for every record); gc (nullable, saturating at 255) and flags as sct_encode. */
int sct_encode_var(int kind, const uint8_t* buf, const int64_t* starts, const int32_t* lens, int64_t n,
                   int words, uint64_t* codes, uint8_t* gc, uint8_t* flags, void* stream);

/* ---------------------------------------------------------------- whitelist ingest
 * Replaces the line loop of Barcodes.from_whitelist (src/sctools/barcode.py:95-97): the
 * file opened 'rb', every line (ending at '\n'; a final line may lack it) chopped by
 * `line[:-1]` (its last byte, whatever it is) and TwoBit-encoded.
 * sct_lines (device, synchronous): starts / lens (the chopped length) of every line; a
 * call with max_lines < the line count only reports *nlines (and *max_len = 0).
 * sct_whitelist_encode_host: the same plus sct_encode_var on the lines, host pointers;
 * call with max_lines = 0 to learn nlines and max_len, then with room for nlines. */
int sct_lines(const uint8_t* d_buf, int64_t nbytes, int64_t max_lines, int64_t* d_starts, int32_t* d_lens,
              int64_t* nlines, int32_t* max_len, void* stream);
/* sct_whitelist_encode (device, ASYNCHRONOUS on stream: no host synchronisation): the same
 * split, chop and encode: a one-read pass for files of 16-base lines (checked on the fly), else a
 * count pass over the file's tiles and an encode pass that numbers the lines from the tile counts;
 * *d_nlines (int64) and *d_maxlen (int32, the longest chopped line) are written on the device;
 * lines g < min(max_lines, *d_nlines) get d_starts[g], d_lens[g], `words` limbs of d_codes,
 * d_gc[g] (nullable) and d_flags[g] (nullable: bit 0 ambiguous, bit 1 invalid byte, bit 2 too long
 * for `words`); rows g >= max_lines are never written, rows in [*d_nlines, max_lines) are
 * unspecified. */
int sct_whitelist_encode(const uint8_t* d_buf, int64_t nbytes, int kind, int words, int64_t max_lines,
                         uint64_t* d_codes, int64_t* d_starts, int32_t* d_lens, uint8_t* d_gc, uint8_t* d_flags,
                         int64_t* d_nlines, int32_t* d_maxlen, void* stream);
int sct_whitelist_encode_host(const uint8_t* buf, int64_t nbytes, int kind, int words, int64_t max_lines,
                              int64_t* nlines, int32_t* max_len, uint64_t* codes, int64_t* starts,
                              int32_t* lens, uint8_t* flags);

/* ---------------------------------------------------------------- decoders
 * TwoBit(L).decode (encodings.py:90-100): exactly L bytes from the LSB upward,
 * bits above 2L ignored.  out: n*L bytes.
 */
int sct_decode2(const uint64_t* codes, int64_t n, int words, int L, uint8_t* out, void* stream);
int sct_decode2_host(const uint64_t* codes, int64_t n, int words, int L, uint8_t* out);
/* ThreeBit.decode (encodings.py:169-180): bytes up to the highest non-zero triplet.
 * out: n*maxlen bytes, record r's sequence right-aligned in its maxlen slot
 * (so it ends at out[(r+1)*maxlen-1]); lengths[r] = its length;
 * bad[r] = -1, or the value (0, 5 or 7) of the lowest-order triplet below the top
 * non-zero one that has no decoding (the reference raises KeyError(value)).
 * maxlen must be >= ceil(64*words/3).
 */
int sct_decode3(const uint64_t* codes, int64_t n, int words, int maxlen, uint8_t* out,
                int32_t* lengths, int32_t* bad, void* stream);
int sct_decode3_host(const uint64_t* codes, int64_t n, int words, int maxlen, uint8_t* out,
                     int32_t* lengths, int32_t* bad);

/* ---------------------------------------------------------------- gc_content
 * TwoBit(L).gc_content (encodings.py:102-111): low bit of each of the L 2-bit groups.
 * ThreeBit.gc_content  (encodings.py:182-192): bit 0 of every triplet of the code.
 * kind 2 uses L; kind 3 ignores it.  out: n int32.
 */
int sct_gc_content(int kind, const uint64_t* codes, int64_t n, int words, int L, int32_t* out,
                   void* stream);
int sct_gc_content_host(int kind, const uint64_t* codes, int64_t n, int words, int L, int32_t* out);

/* ---------------------------------------------------------------- element-wise Hamming
 * TwoBit.hamming_distance (encodings.py:113-121) / ThreeBit.hamming_distance
 * (encodings.py:194-202) of a[r] vs b[r]: number of non-zero 2-bit (3-bit) groups
 * of a^b.  out: n int32.
 */
int sct_hamming_pairs(int kind, const uint64_t* a, const uint64_t* b, int64_t n, int words,
                      int32_t* out, void* stream);
int sct_hamming_pairs_host(int kind, const uint64_t* a, const uint64_t* b, int64_t n, int words,
                           int32_t* out);

/* ---------------------------------------------------------------- scalar server
 * The *_host calls above with n <= 64 records (the drop-in's scalar methods, e.g.
 * TwoBit.encode / hamming_distance, encodings.py:75-121) are served by a resident
 * one-wave kernel per host thread and device that polls a page-locked mailbox, instead of
 * one kernel launch per call; it exits by itself after SCT_TUNE_SCALAR_IDLE_MS (default 5) idle
 * milliseconds and before any kernel that sizes its grid to the resident workgroups.
 * sct_tune_set(SCT_TUNE_SCALAR_SERVER, 0) turns it off (every call is then a launch).
 * sct_scalar_server_stop: ask every server of the process to exit and wait for it.
 * sct_scalar_server_status: server launches so far and servers running now (either may
 * be NULL).
 */
int sct_scalar_server_stop(void);
int sct_scalar_server_status(int64_t* launches, int* running);

/* ---------------------------------------------------------------- all-pairs histogram
 * Replaces the pair loop of Barcodes.summarize_hamming_distances
 * (src/sctools/barcode.py:42-43: itertools.combinations + TwoBit.hamming_distance).
 *
 * A plan holds the bit-sliced selection table of n device-resident uint64 codes
 * (the TwoBit distance is taken over the low `code_bits` bits, code_bits in
 * [1, 64]; every code must be < 2^code_bits).  The unordered pairs i<j are cut
 * into `items` equal work items (row block x column chunk) so that callers can
 * shard them: any partition of [0, items) into ranges, counted on any number of
 * devices and summed, gives the same result.
 *
 * Two count schemes (a plan has one, fixed at creation):
 *
 * SCT_ALLPAIRS_SUBSETS (any code width): sct_allpairs_count ACCUMULATES (atomic add)
 *   ncounts = nbins uint64 "subset counts" into d_counts: d_counts[0] += pairs counted,
 *   d_counts[m] += #pairs whose distance d has all bits of m set (d & m == m),
 *   m = 1..nbins-1.  Every item range is self-contained: its counts invert alone.
 *
 * SCT_ALLPAIRS_MOMENTS (codes of 29..32 bits = 16 bases, the 10x barcode width): the
 *   count kernel accumulates d_counts[0] += pairs and d_counts[1+i] += #pairs whose
 *   d mod 16 has all bits of kMomProducts[i] set (13 products, sct_common.h), and
 *   sct_allpairs_moments accumulates d_counts[14+k-1] += M_k = sum over ALL pairs of
 *   C(16 - d, k), k = 1..3 (pairs agreeing on k chosen positions, from the codes'
 *   position marginals).  ncounts = 17; only the counts of the WHOLE job (every item
 *   counted once, every moment part added once) invert.  13 products instead of 16
 *   cut the count kernel's VALU work per pair.
 *
 * SCT_ALLPAIRS_SPECTRAL (the same 16-base codes): no pair is enumerated.  The histogram
 *   comes from the Walsh-Hadamard transform F of the codes' multiplicity f over Z_2^32:
 *   S_w = sum of F(z)^2 over the z with w non-zero 2-bit digits, w = 0..16, accumulated as
 *   three limbs that never carry (a multiset's sum_w S_w = 2^32 sum f^2 may exceed 2^64):
 *   d_counts[2+w] += bits 0..31, d_counts[19+w] += bits 32..63, d_counts[36+w] += bits 64..
 *   of every partial sum, so S_w = c[2+w] + 2^32 c[19+w] + 2^64 c[36+w]; d_counts[0] += n and
 *   d_counts[1] += sum f^2 (computed from the sorted codes) once, by the range holding item
 *   0.  ncounts = 53.  The host checks S_0 = n^2 and sum_w S_w = 2^32 sum f^2 exactly.
 *   The items are the 2^18 transform slices (z >> 14); the cost of a slice does not
 *   depend on n, so AUTO picks this scheme for large whitelists.  Only
 *   the counts of the whole job invert (host: Krawtchouk transform, checked exact).
 *
 * The counts are linear, so they may be summed across devices (RCCL all-reduce)
 * before sct_counts_to_hist_ex.
 */
typedef struct sct_allpairs_plan sct_allpairs_plan;

#define SCT_ALLPAIRS_AUTO (-1)    /* 16 bases: SPECTRAL from 325K codes, else MOMENTS; else SUBSETS */
#define SCT_ALLPAIRS_SUBSETS 0
#define SCT_ALLPAIRS_MOMENTS 1
#define SCT_ALLPAIRS_SPECTRAL 2

/* Plan flags (sct_allpairs_plan_create_ex2):
 * SCT_ALLPAIRS_DISTINCT  the caller promises pairwise-distinct codes (the keys of a mapping, as
 *   Barcodes.summarize_hamming_distances has them, barcode.py:39-46), so SPECTRAL takes
 *   sum f^2 = n instead of sorting the codes; a broken promise fails the host's exact check
 *   (SCT_E_RANGE), it never yields a histogram. */
#define SCT_ALLPAIRS_DISTINCT 1
/* SCT_ALLPAIRS_NO_CACHE  the plan allocates its own device buffers and frees them when destroyed,
 *   instead of borrowing its device's cached workspace (see sct_allpairs_cache_release). */
#define SCT_ALLPAIRS_NO_CACHE 2

/* = sct_allpairs_plan_create_ex(..., SCT_ALLPAIRS_AUTO, plan) */
int sct_allpairs_plan_create(const uint64_t* d_codes, int64_t n, int code_bits,
                             sct_allpairs_plan** plan);
int sct_allpairs_plan_create_ex(const uint64_t* d_codes, int64_t n, int code_bits, int scheme,
                                sct_allpairs_plan** plan);
/* = sct_allpairs_plan_create_ex with SCT_ALLPAIRS_* flags */
int sct_allpairs_plan_create_ex2(const uint64_t* d_codes, int64_t n, int code_bits, int scheme, int flags,
                                 sct_allpairs_plan** plan);
int sct_allpairs_plan_destroy(sct_allpairs_plan* plan);
/* nbins = max distance + 1 = 2*ceil(code_bits/4)+1; items = number of work items */
int sct_allpairs_plan_info(const sct_allpairs_plan* plan, int* nbins, int64_t* items,
                           int64_t* pairs);
/* scheme of the plan, length of its counts vector, and its code width */
int sct_allpairs_plan_scheme(const sct_allpairs_plan* plan, int* scheme, int* ncounts,
                             int* code_bits);
/* (Re)build the selection table from the codes the plan was created on. */
int sct_allpairs_build(sct_allpairs_plan* plan, void* stream);
/* Build only what counting items [item_begin, item_end) reads (its column chunks; the
 * MOMENTS scheme also re-sorts the codes): a rank of a sharded job calls this with its
 * own item range. */
int sct_allpairs_build_items(sct_allpairs_plan* plan, int64_t item_begin, int64_t item_end,
                             void* stream);
/* Count work items [item_begin, item_end).  grid = 0 picks the persistent grid size. */
int sct_allpairs_count(sct_allpairs_plan* plan, int64_t item_begin, int64_t item_end,
                       uint64_t* d_counts, int grid, void* stream);
/* MOMENTS scheme: add part `part` of `nparts` of the agreement moments to d_counts
 * (the position subsets are split into nparts shares; summing every part once gives
 * M_1..M_3).  SUBSETS scheme: no-op. */
int sct_allpairs_moments(sct_allpairs_plan* plan, int part, int nparts, uint64_t* d_counts,
                         void* stream);
/* Host-only (no device needed): the plan geometry for n codes of code_bits bits, i.e.
 * what sct_allpairs_plan_info would report, plus rows per item and codes per column
 * chunk.  Lets shard drivers partition [0, items) before touching a GPU. */
int sct_allpairs_geometry(int64_t n, int code_bits, int* nbins, int64_t* items, int* rows_per_item,
                          int* cols_per_item);
/* Pairs contained in work items [item_begin, item_end) (host arithmetic; SPECTRAL: the
 * range's share floor(P*end/items) - floor(P*begin/items) of all P pairs). */
int sct_allpairs_range_pairs(const sct_allpairs_plan* plan, int64_t item_begin, int64_t item_end,
                             int64_t* pairs);

/* Bench aid (d_counts receives garbage): the dominant kernel's ms per launch, timed as
 * `repeats` back-to-back launches bracketed by HIP events on `stream`.  SPECTRAL: out[0] =
 * tile kernel, out[1] = seed kernel, both on the first chunk of the range (out[2] = its
 * slices); other schemes: out[0] = count kernel over the range, out[1] = 0, out[2] = items.
 * Needs a built plan. */
int sct_allpairs_time_kernels(sct_allpairs_plan* plan, int64_t item_begin, int64_t item_end,
                              uint64_t* d_counts, int repeats, double* out, void* stream);

/* SPECTRAL plans: bytes per seed value of the seed -> tile intermediate (1, 2 or 4: the
 * densest transform column bounds it), slices per seed / tile launch, codes in the densest
 * column.  Other schemes: SCT_E_INVALID. */
int sct_allpairs_spectral_info(const sct_allpairs_plan* plan, int* elem_bytes, int64_t* chunk_slices,
                               int* max_column);
/* SPECTRAL plans: the transform's column width, 14 (2^18 slices of 2^14 columns) or 16 for sets
 * whose densest 14-bit column needs int16 seeds but whose densest 16-bit column holds <= 127
 * codes (2^16 slices of 2^16 columns, int8 seeds; items stay 2^18 virtual slices, 4 per real
 * slice).  Replaces nothing in the reference (an internal layout choice). */
int sct_allpairs_spectral_columns(const sct_allpairs_plan* plan, int* column_bits);

/* Bench aid: per-launch HIP-event timing of this plan's kernels, recorded on the stream each
 * launch runs on (so it times the launches of a real run, pipelined or not).  mode 1 = start
 * (zeroes the sums), 0 = stop, 2 = read and keep recording.  out (nullable, 8 doubles) =
 * [ms, launches] summed over the recorded launches of kind 0 seed, 1 tile (SPECTRAL), 2 pair
 * count kernel (SUBSETS / MOMENTS), 3 table build (one span per build call); the call waits
 * for the recorded launches. */
int sct_allpairs_timing(sct_allpairs_plan* plan, int mode, double* out);

/* Host: SUBSETS counts -> histogram (exact Moebius inversion), hist[d] for d < nbins. */
int sct_counts_to_hist(const uint64_t* counts, int nbins, uint64_t* hist);
/* Host: counts of any scheme -> histogram (MOMENTS: exact rational solve of the
 * 17 x 17 system; SPECTRAL: Krawtchouk transform; both checked integral and
 * non-negative).  nbins must be the plan's. */
int sct_counts_to_hist_ex(int scheme, const uint64_t* counts, int ncounts, uint64_t* hist,
                          int nbins);

/* One-shot, host pointers, current device: histogram of TwoBit distances over all
 * unordered pairs of the n codes.  hist must hold nbins = 2*ceil(code_bits/4)+1. */
int sct_hamming_hist_allpairs_host(const uint64_t* codes, int64_t n, int code_bits,
                                   uint64_t* hist, int nbins);
/* the same with SCT_ALLPAIRS_DISTINCT.  By default a one-shot call leaves no device memory
 * behind: its plan and staging buffers are its own and freed before it returns (4 GiB for a
 * 16-base set from 325K codes).  sct_keep_workspace(1) keeps them cached per device instead, so
 * repeated calls map nothing (previous: the setting before the call; keep < 0 only reads it). */
int sct_hamming_hist_allpairs_host_ex(const uint64_t* codes, int64_t n, int code_bits, int flags,
                                      uint64_t* hist, int nbins);
int sct_keep_workspace(int keep, int* previous);

/* ---------------------------------------------------------------- several devices, one process
 * SURVEY §8(b) `n_gpus` (sct_init(n_gpus) / an n_gpus argument in the survey's sketch): the
 * one-shot and host-stream calls split across devices[0..ndev) of this process (HIP ordinals;
 * repeats are logical shards of one GPU).  Slot r runs on a persistent worker thread of its own
 * with devices[r] current; the calling thread's current device is not changed.  devices == NULL
 * or ndev == 1: the single-device call on the current device (or devices[0]).  One multi-device
 * call runs at a time per process (calls from several threads queue).
 *
 * All-pairs (replaces barcode.py:42-43 like sct_hamming_hist_allpairs_host_ex): every slot holds
 * a replica of the codes and counts the item range items*r/ndev .. items*(r+1)/ndev (SPECTRAL:
 * transform slices) plus moment part r of ndev; the 53 / 17 / nbins counts of the slots are summed
 * on the host -- where they are needed anyway -- and inverted once.  Bit-identical for any ndev. */
int sct_hamming_hist_allpairs_host_devices(const uint64_t* codes, int64_t n, int code_bits, int flags,
                                           const int* devices, int ndev, uint64_t* hist, int nbins);
/* Nearest whitelist: contiguous query ranges per slot, the whitelist indexed on every device
 * (no exchange).  The multi plan keeps one index per slot for a stream of query batches. */
int sct_nearest_host_devices(int kind, const uint64_t* whitelist, int64_t nw, const uint64_t* queries, int64_t nq,
                             int code_bits, int max_d, const int* devices, int ndev, int32_t* index,
                             uint8_t* dist);
typedef struct sct_nearest_multi sct_nearest_multi;
int sct_nearest_multi_create_host(int kind, const uint64_t* whitelist, int64_t nw, int code_bits, int max_d,
                                  const int* devices, int ndev, sct_nearest_multi** plan);
int sct_nearest_multi_query_host(sct_nearest_multi* plan, const uint64_t* queries, int64_t nq, int32_t* index,
                                 uint8_t* dist);
int sct_nearest_multi_destroy(sct_nearest_multi* plan);
/* Host encode stream (sct_encode_stream_host) over contiguous record ranges, one per slot. */
int sct_encode_stream_host_devices(int kind, const uint8_t* seqs, int64_t n, int L, uint64_t* codes, uint8_t* gc,
                                   uint8_t* flags, int64_t chunk, const int* devices, int ndev);

/* Plan cache: a plan created while no other plan holds its device's cached buffers borrows
 * them (the SPECTRAL intermediate of up to 4 GiB, codes, bit planes, order table) and leaves
 * them allocated when destroyed, so repeated one-shot calls map no device memory (the
 * drop-in's summarize_hamming_distances, barcode.py:39-46, is one such call).  This frees
 * every idle cache (all devices); a cache lent to a live plan is freed when that plan is
 * destroyed.  sct_tune_set(SCT_TUNE_PLAN_CACHE, 0) turns the cache off.  The idle memory of
 * the library's stream-ordered scratch pool (host-stream stages, ingest scratch) is trimmed
 * too, after a synchronisation of the current device, and the calling thread's staging buffer
 * on the current device is freed. */
int sct_allpairs_cache_release(void);

/* ---------------------------------------------------------------- all-pairs, wide codes
 * The same pair loop (barcode.py:42-43) for keys of any width up to 256 limbs: codes are
 * n x `words` little-endian uint64 limbs (Python ints >= 2^64: ThreeBit-encoded 22..28-bp
 * barcodes, TwoBit > 32 bp).  TwoBit.hamming_distance (encodings.py:113-121) of multi-limb
 * codes = the sum of the per-limb counts (no 2-bit group straddles a limb).  Work items
 * are pairs of 256-code tiles (a <= b, row-major), so contiguous item ranges shard across
 * devices; sct_allpairs_wide ACCUMULATES hist[d] (nbins = 32 * words + 1 uint64) with
 * the pairs i < j of items [item_begin, item_end). */
int sct_allpairs_wide_geometry(int64_t n, int words, int64_t* items, int* nbins);
int sct_allpairs_wide_range_pairs(int64_t n, int64_t item_begin, int64_t item_end, int64_t* pairs);
int sct_allpairs_wide(const uint64_t* d_codes, int64_t n, int words, int64_t item_begin, int64_t item_end,
                      uint64_t* d_hist, int nbins, void* stream);
int sct_hamming_hist_allpairs_wide_host(const uint64_t* codes, int64_t n, int words, uint64_t* hist,
                                        int nbins);

/* ---------------------------------------------------------------- base frequency
 * Replaces Barcodes.base_frequency (src/sctools/barcode.py:48-70): out[p*4 + v] =
 * number of codes whose base p (0 = first, MSB-first TwoBit packing) has 2-bit value
 * v (A 0, C 1, T 2, G 3); bases above bit 63 read as 0, as the reference's uint64
 * keys >>= 2 loop does.  out: L*4 uint64, overwritten.  L <= 1024.
 */
int sct_base_frequency(const uint64_t* codes, int64_t n, int L, uint64_t* out, void* stream);
int sct_base_frequency_host(const uint64_t* codes, int64_t n, int L, uint64_t* out);

/* ---------------------------------------------------------------- nearest whitelist
 * No reference function exists; the contract is the brute-force
 * composition of the reference's distance (kind 2: TwoBit.hamming_distance,
 * encodings.py:113-121; kind 3: ThreeBit.hamming_distance, encodings.py:194-202):
 *   index[i] = j  if exactly one whitelist index j attains d_min(q_i) <= max_d,
 *            = -2 if several indices attain it, -1 if d_min > max_d;
 *   dist[i]  = d_min if <= max_d, else 255.
 * The plan is an exact pigeonhole index (max_d <= 1 on A/C/G/T whitelists: half-key tables;
 * otherwise open-addressing or CSR buckets per position block); it copies nothing from the
 * caller after create returns (the whitelist is bucketed).  A half-key whitelist sorted
 * alphabetically, or numerically as TwoBit or ThreeBit codes, is queried in one kernel (table
 * position = whitelist index); any other order adds a pass mapping positions to indices.  The
 * answers never depend on the order.
 * code_bits: bits covered by the block split (whitelist codes < 2^code_bits).
 */
typedef struct sct_nearest_plan sct_nearest_plan;
int sct_nearest_plan_create(int kind, const uint64_t* d_whitelist, int64_t nw, int code_bits,
                            int max_d, void* stream, sct_nearest_plan** plan);
int sct_nearest_plan_destroy(sct_nearest_plan* plan);
int sct_nearest_query(sct_nearest_plan* plan, const uint64_t* d_queries, int64_t nq,
                      int32_t* d_index, uint8_t* d_dist, void* stream);
/* the index layout the plan chose and its device bytes */
#define SCT_NEAREST_OA 1       /* open-addressing tables of block-pair keys */
#define SCT_NEAREST_CSR 2      /* CSR buckets per block */
#define SCT_NEAREST_HALVES 3   /* sorted half-key tables (max_d <= 1, ACGT whitelists) */
int sct_nearest_plan_info(const sct_nearest_plan* plan, int* scheme, int64_t* index_bytes);
int sct_nearest_host(int kind, const uint64_t* whitelist, int64_t nw, const uint64_t* queries,
                     int64_t nq, int code_bits, int max_d, int32_t* index, uint8_t* dist);
/* A plan from a HOST whitelist (copied for the build, not kept), and queries from host memory
 * against it: a stream of batches builds the index once (barcode.WhitelistCorrector).  The
 * query call copies the queries in, runs sct_nearest_query on the thread's stream with scratch
 * from the library's stream-ordered pool, and returns with index / dist in host memory
 * (page-locked buffers are copied by DMA in place). */
int sct_nearest_plan_create_host(int kind, const uint64_t* whitelist, int64_t nw, int code_bits, int max_d,
                                 sct_nearest_plan** plan);
int sct_nearest_query_host(sct_nearest_plan* plan, const uint64_t* queries, int64_t nq, int32_t* index,
                           uint8_t* dist);

/* ---------------------------------------------------------------- FASTQ barcode extraction
 * Replaces the per-record path reader.Reader.__iter__ (src/sctools/reader.py:56-85) ->
 * fastq.Reader.record_grouper (src/sctools/fastq.py:143-150) -> Record name check
 * (fastq.py:31-38) -> EmbeddedBarcodeGenerator / extract_barcode (fastq.py:181-200):
 * record.sequence[start:end] and record.quality[start:end] of every record.
 * The input is the files' bytes concatenated (file_ends = cumulative end offsets, the last
 * == nbytes; a record may span files, an incomplete trailing record is dropped).  Lines
 * keep their newline, so slices of short reads include '\n' exactly as in Python.
 * text_mode = 0 is open(..., 'rb'): lines end at '\n'; 1 is 'r': '\n', "\r\n" and a lone
 * '\r' each end a line and read back as '\n' (ASCII input only, else SCT_E_RANGE).
 * first_bad_name = the first record whose name line does not start with '@' (the
 * reference raises ValueError('fastq name must start with @') there), or -1.
 */
typedef struct sct_fastq_index sct_fastq_index;
/* Pass 1: count every 4 KiB tile's lines (-> nrecords = lines / 4); keeps only per-tile
 * line offsets.  The buffer must stay alive and unchanged until the index is destroyed. */
int sct_fastq_index_create(const uint8_t* d_buf, int64_t nbytes, const int64_t* file_ends, int nfiles,
                           int text_mode, void* stream, sct_fastq_index** index);
int sct_fastq_index_destroy(sct_fastq_index* index);
/* first_bad_name: from the last sct_fastq_extract_spans (-2 before any). */
int sct_fastq_index_info(const sct_fastq_index* index, int64_t* nrecords, int64_t* nlines,
                         int64_t* first_bad_name);
/* Pass 2, synchronous: every record's sequence-line and quality-line slices for all spans
 * (nspans <= 8 host (start, end) pairs, end <= 4096) and the '@' check of every name line.
 * Span k's rows start at d_seq / d_qual + nrecords * sum_{i<k} width_i (zero padded rows of
 * width_k), lengths at d_seq_len / d_qual_len + k * nrecords; every output is nullable. */
int sct_fastq_extract_spans(sct_fastq_index* index, const uint8_t* d_buf, const int32_t* spans,
                            int nspans, uint8_t* d_seq, uint8_t* d_qual, int32_t* d_seq_len,
                            int32_t* d_qual_len, int64_t* first_bad_name, void* stream);
/* Index and extraction in one call (a count pass, then the extraction; asynchronous on
 * `stream`, no host synchronisation): d_file_ends is DEVICE memory; rows are laid out by the
 * caller's capacity (span k's row r at out + cap_records * prefix_k + r * width_k; lengths at
 * len + k * cap + r; records >= cap_records are not written); d_status (3 int64, device): [0]
 * line count (records = lines / 4), [1] ~(first bad-name record) or 0, [2] non-ASCII seen (text
 * mode rejects it).  d_codes0 / d_gc0 / d_flags0 (nullable): span 0's sequence rows encoded as
 * sct_encode(code_kind) would encode those rows (code_kind 2 TwoBit, width <= 32; 3 ThreeBit,
 * width <= 21 -- N kept, the queries of sct_nearest_query). */
int sct_fastq_extract_fused(const uint8_t* d_buf, int64_t nbytes, const int64_t* d_file_ends, int nfiles,
                            int text_mode, const int32_t* spans, int nspans, int64_t cap_records, uint8_t* d_seq,
                            uint8_t* d_qual, int32_t* d_seq_len, int32_t* d_qual_len, uint64_t* d_codes0,
                            uint8_t* d_gc0, uint8_t* d_flags0, int code_kind, int64_t* d_status, void* stream);
/* Host convenience: spans = nspans (start, end) pairs.  Call with max_records < the record
 * count to learn nrecords (outputs untouched); then with room for nrecords:
 * seq_out/qual_out (nullable) = span k's rows at offset sum_{i<k} nrecords*width_i,
 * seq_len/qual_len (nullable) = nspans x nrecords lengths. */
int sct_fastq_extract_host(const uint8_t* buf, int64_t nbytes, const int64_t* file_ends, int nfiles,
                           int text_mode, const int32_t* spans, int nspans, uint8_t* seq_out,
                           uint8_t* qual_out, int32_t* seq_len, int32_t* qual_len,
                           int64_t max_records, int64_t* nrecords, int64_t* first_bad_name);

/* Streaming form (reader.Reader reads its files lazily, reader.py:56-85): a stream keeps
 * its device buffers across pieces of the concatenated files.  Each piece must end on a
 * '\n' unless final; file_ends are the files' ends inside the piece (the last == nbytes).
 * chunk: extracts every complete record of the piece on the device; consumed = the byte
 * just past the last complete record (final = 1: nbytes, the incomplete tail dropped);
 * the caller starts the next piece there.  fetch: that piece's outputs, laid out as
 * sct_fastq_extract_host's (each nullable; qualities only if the stream keeps them). */
typedef struct sct_fastq_stream sct_fastq_stream;
int sct_fastq_stream_create(int text_mode, const int32_t* spans, int nspans, int qualities,
                            sct_fastq_stream** stream);
int sct_fastq_stream_destroy(sct_fastq_stream* stream);
int sct_fastq_stream_chunk(sct_fastq_stream* stream, const uint8_t* buf, int64_t nbytes, const int64_t* file_ends,
                           int nfiles, int final, int64_t* nrecords, int64_t* consumed, int64_t* first_bad_name);
int sct_fastq_stream_fetch(sct_fastq_stream* stream, uint8_t* seq_out, uint8_t* qual_out, int32_t* seq_len,
                           int32_t* qual_len);
/* Copy the NEXT piece to the device ahead of its chunk call (asynchronous, on a copy stream of
 * the stream's own): a caller that knows the next piece while it works on this one's results
 * overlaps the piece's PCIe copy with that work.  Only a page-locked piece (sct_host_pinned) is
 * staged (anything else: a no-op); the piece's bytes must stay unchanged until the chunk call
 * for exactly (buf, nbytes) -- which then skips its own copy -- or the next stage call, or
 * the stream's destruction (each waits for the copy). */
int sct_fastq_stream_stage(sct_fastq_stream* stream, const uint8_t* buf, int64_t nbytes);

/* ---------------------------------------------------------------- bench aid
 * Streaming device copy (16 B per lane, nontemporal, resident grid) of `bytes` (a multiple
 * of 16): the practical HBM ceiling bench.py prices the kernels against beside the spec. */
int sct_stream_copy(void* d_dst, const void* d_src, int64_t bytes, void* stream);

/* ---------------------------------------------------------------- summary
 * Replaces barcode.py:44-46 (np.percentile(distances,[0,25,50,75,100]) with numpy's
 * default 'linear' method, then np.mean) computed from the histogram alone,
 * bit-exact in float64.  out[0..5] = minimum, 25th percentile, median,
 * 75th percentile, maximum, average.  Returns SCT_E_RANGE when the histogram is
 * empty (the reference raises IndexError).
 */
int sct_summary_from_hist(const uint64_t* hist, int nbins, double* out);

#ifdef __cplusplus
}
#endif

#endif /* SCTOOLS_HIP_H */
