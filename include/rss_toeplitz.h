/*
 * rss_toeplitz.h -- C ABI of the MI355X (gfx950) RSS Toeplitz hashing engine.
 *
 * This is the drop-in boundary for the reference's hot path.  The reference
 * (noamsto/rss_simulator_nvidia v0.0.2) is pure Python and has no FFI, so each
 * entry point below names the Python function whose job it takes over; the
 * Python mirror in rss_simulator_nvidia_amd/ binds them through ctypes
 * (rss_simulator_nvidia_amd/_native.py) and INTEGRATION.md shows the ctypes stub
 * a reference maintainer would add.
 *
 * Conventions
 *   - plain C types only; buffers are caller-owned; nothing here allocates on
 *     behalf of the caller except an rss_ctx (which owns its device scratch);
 *   - every function returns RSS_OK (0) or a negative errno-style code and never
 *     aborts; rss_last_error() returns a thread-local message for the last
 *     failure on the calling thread;
 *   - "device" entry points take device pointers and a hipStream_t passed as
 *     void* (NULL = the legacy default stream) and are stream-ordered: they
 *     enqueue work and return without synchronising;
 *   - all arithmetic is integer and bit-exact to the reference.
 */
#ifndef RSS_TOEPLITZ_H
#define RSS_TOEPLITZ_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RSS_ABI_VERSION 1

/* status codes (negative errno values) */
#define RSS_OK 0
#define RSS_EIO (-5)      /* HIP runtime / device failure                         */
#define RSS_ENOMEM (-12)  /* device or pinned allocation failed                   */
#define RSS_EINVAL (-22)  /* bad argument (NULL, bad key length, zero htable ...) */
#define RSS_ENODEV (-19)  /* no usable gfx950 device                              */
#define RSS_ENOTSUP (-95) /* CSV not in the canonical fast-path form (use pandas)  */

/*
 * One IPv4 4-tuple, packed to 12 bytes, 4-byte aligned.  The three host-order
 * words are exactly the 96-bit big-endian Toeplitz input of
 * rss_simulator/toeplitz.py:113-142 (__prepare_input_bytes): src_ip, dst_ip,
 * then (src_port & 0xFFFF) << 16 | (dst_port & 0xFFFF).  Ports are masked to 16
 * bits by the caller, matching toeplitz.py:138-141.
 */
typedef struct rss_tuple4 {
    uint32_t sip;
    uint32_t dip;
    uint32_t ports;
} rss_tuple4;

#define RSS_KEY_MIN_BYTES 4
#define RSS_KEY_MAX_BYTES 52
#define RSS_INPUT_BITS 96

/*
 * Prepared hash key.  window[i] is the 32-bit window the reference XORs in
 * for input bit i (toeplitz.py:65-68 with __key_left_most_32bits :71-81 after i
 * rotations by __shift_key :83-98), i.e. key bits [i, i+32) MSB-first (bit
 * indices taken modulo 8*len, which only matters for keys shorter than 16
 * bytes).  The device kernel expands the windows into its LDS lookup tables.
 * For len >= 16 only key bytes 0..15 influence any hash.
 */
typedef struct rss_key {
    uint32_t len;                          /* key length in bytes (>= 4)     */
    uint8_t bytes[RSS_KEY_MAX_BYTES];      /* first min(len, 52) key bytes   */
    uint32_t window[RSS_INPUT_BITS];
} rss_key;

/*
 * Replaces HashKey.__from_str's conversion result -> Toeplitz(key)
 * (rss_simulator/hash_key.py:12-32, rss_simulator/toeplitz.py:8-15).  `key`
 * holds `len` raw bytes, len >= 4.  The CLI's key regex admits only 40 or 52
 * (hash_key.py:25-28), but Toeplitz(list) accepts any list of >= 4 bytes, and a
 * key shorter than 16 bytes wraps during the rotation -- reproduced here.  Text
 * parsing stays in the caller.
 */
int rss_key_prepare(const uint8_t* key, size_t len, rss_key* out);

/*
 * Field selection (the reference's planned "select what
 * will be the fields used for the RSS function", docs/rss_general_explaination.md:14-18,
 * i.e. ethtool's rx-flow-hash s/d/f/n).  The hash input becomes the concatenation
 * of the selected fields in the order src_ip, dst_ip, src_port, dst_port.  Since
 * Toeplitz is linear in the input bits, that equals hashing the full 12-byte tuple
 * with window[i] replaced by the window of bit i's position in the concatenation
 * (0 for unselected bits): the kernel is unchanged.  Apply once, after
 * rss_key_prepare.  RSS_FIELDS_IP is the "IPv4 only" hash of the Microsoft RSS
 * verification suite.
 */
#define RSS_FIELD_SRC_IP 1u
#define RSS_FIELD_DST_IP 2u
#define RSS_FIELD_SRC_PORT 4u
#define RSS_FIELD_DST_PORT 8u
#define RSS_FIELDS_IP (RSS_FIELD_SRC_IP | RSS_FIELD_DST_IP)
#define RSS_FIELDS_ALL 15u
int rss_key_select_fields(rss_key* key, uint32_t fields);

/* flags for rss_hash_device / rss_hash_host */
#define RSS_FLAG_ACCUMULATE 1u  /* add into counts instead of overwriting them      */
#define RSS_FLAG_QUEUE_U16 2u   /* rss_hash_device: d_queue is uint16_t[n] (Q<=2^16) */
#define RSS_FLAG_QUEUE_U8 4u    /* rss_hash_device: d_queue is uint8_t[n]  (Q<=256)  */
/* rss_hash_device: 64-bit addressing even where every stream's byte offsets fit 32 bits
 * (the instance batches of >= 2^32 / 12 tuples run).  Same results and the same access
 * shape; it only gives the launch a kernel symbol of its own in traces -- the placement
 * probe and the clock settle use it, so a profile's row for the 32-bit instance holds the
 * resident step's launches alone. */
#define RSS_FLAG_ADDR64 8u

/*
 * Device-resident hot path.  Replaces, for n tuples at once:
 *   Simulator.calc_hash          rss_simulator/simulator.py:74-92
 *     -> Toeplitz.compute_hash    rss_simulator/toeplitz.py:46-69
 *   Simulator.calc_queue_number  rss_simulator/simulator.py:94-98
 *     (queue = hash % htable % nqueues)
 *   the value_counts of Simulator.write_statistics  simulator.py:107-113
 *     (counts[q] = number of tuples with queue q, for q < nqueues).
 * d_tuples: n packed tuples in device memory.  d_hash: n uint32 or NULL.
 * d_queue: n queue numbers or NULL -- uint32 by default, uint16 / uint8 with
 * RSS_FLAG_QUEUE_U16 / RSS_FLAG_QUEUE_U8 (same values, narrower stores; the flag is
 * rejected if the queues do not fit).  Every queue is < min(htable, nqueues) (bucket <
 * htable), so bins, the width check and the counts the kernel writes are sized by
 * min(htable, nqueues): --num-queues 4e9 with htable 128 fits a u8 column and 128 bins.
 * d_counts: nqueues uint64 or NULL; overwritten unless RSS_FLAG_ACCUMULATE (entries
 * [min(htable, nqueues), nqueues) are then zero -- callers may size counts by
 * min(htable, nqueues) and pass that as nqueues).  htable >= 1, nqueues >= 1
 * (positive_int.py:27).  Launched on `stream` (hipStream_t) on the calling
 * thread's current device.  Any alignment works; 16-byte aligned tuples/hashes
 * (and 4/8/16-byte aligned u8/u16/u32 queues) take the 4-tuples-per-lane path.
 * Counts-only launches with a power-of-two htable <= 256 run a table-free kernel;
 * with more than 8192 queues the counts go to guarded LDS bins of the hash pass itself --
 * u16 bins for up to 16384 queues beside the 12-bit tables and up to 80572 beside the
 * 2.6 KiB small tables (4-tuple body, no indirection table), u8 bins for up to 161144 --
 * whose per-workgroup rows a reduce launch sums; the queues past that are counted by wide
 * passes (163840 queues per pass in u8 bins, 65536 in u16) over d_queue when given, else --
 * counts only -- over per-wave lists of the tuples whose queue lies past the LDS range (the
 * queue minus 161144, 2 bytes per entry for nqueues <= 226680, else 4).  A guarded bin that
 * wraps (a batch piling many tuples onto one queue at once) poisons its pass and a gated
 * recount with u32 bins replaces that pass's counts: exact for any input.  Scratch for the
 * rows, the lists and the passes is stream-ordered hipMallocAsync / hipFreeAsync on
 * `stream`, all of it taken before the first pass touches d_counts; a launch that cannot
 * get it counts with one global atomic per tuple instead (same counts, slower), as it does
 * when a guarded path would need more narrow passes than the atomics cost.
 */
int rss_hash_device(const rss_key* key, const rss_tuple4* d_tuples, size_t n,
                    uint32_t htable, uint32_t nqueues, uint32_t* d_hash,
                    void* d_queue, uint64_t* d_counts, uint32_t flags,
                    void* stream);

/*
 * Single-pass counts: rss_hash_device with a caller-owned workspace, so that a batch's
 * counts need no zeroing launch before it (the step of a job that hashes batch after
 * batch into fresh counts, sharding.CountsPipeline).  Every workgroup adds, for every
 * queue, its bin total plus one arrival (1 << 44) into the workspace; the add that sees the
 * last arrival writes that queue's count into d_counts -- overwriting it, or adding with
 * RSS_FLAG_ACCUMULATE -- and zeroes its word again.  d_workspace: rss_counts_workspace_bytes(nqueues) bytes of 8-byte
 * aligned device memory (one word per queue + the balanced tail's unit counter + one spare),
 * zero before its first use (every launch leaves it zero), used
 * by one launch at a time (launches that may run concurrently need their own).  Launches
 * whose counts are not gathered in private/shared LDS bins (more than 8192 queues) leave the workspace
 * untouched and zero d_counts first as rss_hash_device does.  Results are identical to
 * rss_hash_device's.  With d_counts NULL the workspace is not used (may be NULL).
 * Ordering: a queue's count travels in the atomics on its own word, and the balanced
 * tail's counter (below) is reset by the launch's final claim on it, so no fence is needed
 * (the memory model's single-location coherence); stress-tested in
 * tests/test_gpu_single_pass.py.  Launches of >= 2^24 tuples
 * also take the last tenth of their work from a counter in the workspace (the balanced tail: the XCDs finish
 * together), so a workspace must never be shared by two launches in flight.
 */
int rss_counts_workspace_bytes(uint32_t nqueues, size_t* out);
int rss_hash_device_ws(const rss_key* key, const rss_tuple4* d_tuples, size_t n,
                       uint32_t htable, uint32_t nqueues, uint32_t* d_hash,
                       void* d_queue, uint64_t* d_counts, uint32_t flags,
                       uint64_t* d_workspace, void* stream);

/*
 * Indirection table (RETA; `ethtool -X equal N / weight ...`, which the reference's
 * docs cite, docs/rss_general_explaination.md:9-11): queue = reta[hash % htable]
 * instead of (hash % htable) % nqueues.  reta: host array of htable entries, each
 * < nqueues; htable <= 1024.  The reference's mapping is the table reta[b] = b %
 * nqueues ("equal").  Everything else as rss_hash_device / rss_hash_host.
 */
int rss_hash_device_reta(const rss_key* key, const rss_tuple4* d_tuples, size_t n,
                         uint32_t htable, const uint32_t* reta, uint32_t nqueues,
                         uint32_t* d_hash, void* d_queue, uint64_t* d_counts, uint32_t flags,
                         void* stream);

/*
 * Synthetic input: tuple i (i = first_index .. first_index+n-1) is
 *   r0 = mix64(seed + 2i), r1 = mix64(seed + 2i + 1)       (mod 2^64)
 *   sip = r0 >> 32, dip = (uint32)r0, ports = (uint32)r1
 * with mix64 the splitmix64 finaliser (gamma 0x9E3779B97F4A7C15).  The oracle
 * restates the same generator, so any shard can be rebuilt on the host.
 */
int rss_generate_tuples(uint64_t seed, uint64_t first_index, size_t n,
                        rss_tuple4* d_tuples, void* stream);

/*
 * Key search (the reference's random_hash_key,
 * hash_key.py:53-60, is the candidate generator this evaluates at scale): for
 * each of nkeys keys, the per-queue counts of the same n device-resident tuples.
 * d_windows: nkeys x 96 uint32 in device memory, key k's rss_key::window at
 * k*96.  d_counts: nkeys x nqueues uint64, row k = key k, overwritten.  One
 * launch; each workgroup builds one key's tables and histograms a slice.
 */
int rss_key_search_device(const uint32_t* d_windows, size_t nkeys,
                          const rss_tuple4* d_tuples, size_t n, uint32_t htable,
                          uint32_t nqueues, uint64_t* d_counts, void* stream);

/*
 * IPv6.  36-byte input = src addr (16 B) | dst addr (16 B) |
 * src port | dst port, the layout of the Microsoft RSS IPv6 hash; stored as nine
 * host-order words whose big-endian bytes are that input (w[0..3] src, w[4..7]
 * dst, w[8] = sport << 16 | dport).  288 input bits use key bits up to 319, which
 * a 40-byte key covers without wrapping.  Fields for rss_key6_select_fields use
 * the same RSS_FIELD_* bits (RSS_FIELDS_IP = the "IPv6 only" hash).  Flags as for
 * rss_hash_device (d_queue holds uint32, or uint16 / uint8 with RSS_FLAG_QUEUE_U16 /
 * RSS_FLAG_QUEUE_U8); rss_hash6_host writes uint32 queues.
 */
#define RSS_INPUT6_BITS 288
typedef struct rss_tuple6 {
    uint32_t w[9];
} rss_tuple6;

typedef struct rss_key6 {
    uint32_t len;
    uint32_t window[RSS_INPUT6_BITS];
} rss_key6;

int rss_key6_prepare(const uint8_t* key, size_t len, rss_key6* out);
int rss_key6_select_fields(rss_key6* key, uint32_t fields);
int rss_hash6_device(const rss_key6* key, const rss_tuple6* d_tuples, size_t n,
                     uint32_t htable, uint32_t nqueues, uint32_t* d_hash, void* d_queue,
                     uint64_t* d_counts, uint32_t flags, void* stream);
/* rss_hash6_device with single-pass counts, as rss_hash_device_ws: d_workspace is a zeroed,
 * 8-byte aligned device buffer of rss_counts_workspace_bytes(nqueues) bytes used by one launch
 * at a time (every launch leaves it zero); the kernel's last workgroup writes the counts, so
 * no zeroing launch runs before it, and launches of >= 2^24 tuples hand their last rows out
 * per workgroup slot (the balanced tail) -- the IPv6 counterpart of the IPv4 bench step. */
int rss_hash6_device_ws(const rss_key6* key, const rss_tuple6* d_tuples, size_t n,
                        uint32_t htable, uint32_t nqueues, uint32_t* d_hash, void* d_queue,
                        uint64_t* d_counts, uint32_t flags, uint64_t* d_workspace, void* stream);

/*
 * Host-memory convenience path (CSV in -> CSV out): owns device buffers.
 * Thread safety: any number of host threads may call the entry points that take one
 * context at once; each call holds the context's lock from entry to return, so calls on
 * one context run one after another (each with its own results) and calls on different
 * contexts run concurrently.  Replaces the reentrancy of the reference's per-call
 * Toeplitz.compute_hash (rss_simulator/toeplitz.py:59 copies the key on every call).
 * rss_ctx_destroy must not race a call on the same context.  Output that a call leaves in
 * context-owned memory (rss_csv_hash_text's file image) is valid until the next call on
 * that context, whichever thread makes it.  A call that fails returns only after every
 * copy and kernel it queued has finished: the caller's buffers are its own again.
 */
typedef struct rss_ctx rss_ctx;

int rss_ctx_create(int device, rss_ctx** out);
void rss_ctx_destroy(rss_ctx* ctx);

/*
 * Same contract as rss_hash_device but on host buffers: chunked
 * H2D -> kernel -> D2H through pinned staging, synchronous on return.
 * h_hash / h_queue (uint32) / h_counts may be NULL; only RSS_FLAG_ACCUMULATE
 * is honoured.  Buffers that are already page-locked (rss_host_alloc,
 * hipHostMalloc, hipHostRegister) are copied by DMA directly, without the
 * staging copy; pageable buffers go through the context's pinned staging.
 */
int rss_hash_host(rss_ctx* ctx, const rss_key* key, const rss_tuple4* h_tuples,
                  size_t n, uint32_t htable, uint32_t nqueues, uint32_t* h_hash,
                  uint32_t* h_queue, uint64_t* h_counts, uint32_t flags);

/*
 * Page-locked host memory for rss_hash_host's direct-DMA path (hipHostMalloc).
 * Pinning costs far more than a copy, so allocate once and reuse across batches.
 * rss_host_free(NULL) is a no-op.
 */
int rss_host_alloc(size_t bytes, void** out);
void rss_host_free(void* p);

/*
 * ---- CSV fast path (host, multi-threaded) ----
 * Replaces pd.read_csv (rss_simulator/simulator.py:55) and the two to_csv calls
 * of write_statistics (simulator.py:114-115) for CANONICAL files: header = the
 * four columns src_ip,dst_ip,src_port,dst_port in any order and nothing else;
 * rows = four unquoted fields, dotted-quad addresses with octets 0..255 and no
 * leading zeros, ports 0..65535 in plain decimal; LF or CRLF; empty lines
 * skipped; ASCII only.  pandas round-trips such fields unchanged, so the output
 * is byte-identical to the reference's.  Any other file -> RSS_ENOTSUP: the
 * caller must take the pandas path, which reproduces the reference's parsing
 * and error behaviour.  `threads` <= 0 picks min(16, hardware threads).
 */
typedef struct rss_csv_layout {
    uint8_t field_column[4]; /* field f of a row holds column field_column[f]:
                                0 src_ip, 1 dst_ip, 2 src_port, 3 dst_port   */
} rss_csv_layout;

/* Parse the whole file image; RSS_EINVAL with *n_rows set if cap is too small. */
int rss_csv_parse(const char* data, size_t len, rss_tuple4* tuples, size_t cap,
                  size_t* n_rows, rss_csv_layout* layout, int threads);

/* Upper bound of rss_csv_format's output size. */
size_t rss_csv_format_bound(size_t n, uint32_t nqueues);

/*
 * An address column of a DataFrame (Simulator.calc_hash on pandas data, whatever file or
 * frame it came from): `text` holds its n cells joined by '\n'.  Cell i that is a plain
 * quad -- four dot-separated runs of 1-3 ASCII digits, nothing else -- gets ok[i] = 1 (2 when
 * it is also canonical: octets 0..255 without leading zeros, the text rss_csv_format writes
 * back, so a write_statistics of such cells may take the native formatter) and
 * out[i] = (o0 << 24 | o1 << 16 | o2 << 8 | o3) mod 2^32 with the octets NOT range-checked
 * and OR-combined, exactly __ip_to_int + the byte masks of __prepare_input_bytes
 * (rss_simulator/toeplitz.py:100-111, :127-137); any other cell gets ok[i] = 0 and the caller
 * converts it with the reference's own rules (whitespace, extra octets, errors).  RSS_EINVAL
 * when the text does not hold exactly n cells (a cell containing '\n').
 */
int rss_parse_dotted(const char* text, size_t len, size_t n, uint32_t* out, uint8_t* ok);

/*
 * The same for an IPv6 address column (the additive --ipv6 input): cell i that is RFC 4291
 * text without an embedded IPv4 part or zone (1-4 hex digits per group, at most one '::';
 * the CSV path's canonical IPv6 form) gets ok[i] = 1 and out[4i..4i+3] = its 128 bits as four
 * big-endian-valued words, as ipaddress.IPv6Address reads it; any other cell ok[i] = 0.
 */
int rss_parse_ipv6(const char* text, size_t len, size_t n, uint32_t* out, uint8_t* ok);

/*
 * Write the statistics file of write_statistics (simulator.py:100-115): the
 * "queue_number,counts" rows of the non-empty queues, then the table with the
 * input columns in input order plus hash_result,queue_number.  `cap` must be
 * >= rss_csv_format_bound(n, nqueues).
 */
int rss_csv_format(const rss_tuple4* tuples, const uint32_t* hash, const uint32_t* queue,
                   size_t n, const uint64_t* counts, uint32_t nqueues,
                   const rss_csv_layout* layout, char* out, size_t cap, size_t* out_len,
                   int threads);

/*
 * IPv6 rows through the same fast path (the --ipv6 input of SURVEY.md §8f row 4;
 * pandas path: Simulator with ipv6, ingest.pack_frame6).  Canonical IPv6 fields are
 * RFC 4291 text without an embedded IPv4 part or zone id (1-4 hex digits per group,
 * at most one "::"); ports and the header as above.  rss_csv_parse6 fills tuples[n]
 * and spans[2n] (byte offsets of each row's text, line end excluded); pandas keeps
 * the address strings verbatim, so rss_csv_format6 writes each row as its input text
 * + ",hash,queue" after the same counts prefix.  Same return codes as the IPv4 pair.
 */
int rss_csv_parse6(const char* data, size_t len, rss_tuple6* tuples, uint64_t* spans, size_t cap,
                   size_t* n_rows, rss_csv_layout* layout, int threads);
size_t rss_csv_format6_bound(const uint64_t* spans, size_t n, uint32_t nqueues);
int rss_csv_format6(const char* data, const uint64_t* spans, const uint32_t* hash,
                    const uint32_t* queue, size_t n, const uint64_t* counts, uint32_t nqueues,
                    const rss_csv_layout* layout, char* out, size_t cap, size_t* out_len,
                    int threads);

/*
 * ---- CSV on the device ----
 * The whole `--csv` job for a CANONICAL file image (the rules above): the body goes
 * to the device once, newlines are indexed, rows parsed, hashed (rss_hash_device or,
 * with `reta`, rss_hash_device_reta), and the statistics file of write_statistics is
 * formatted there; the header and per-queue count lines are built on the host.
 * Replaces pd.read_csv (simulator.py:55), calc_hash / calc_queue_number (:74-98)
 * and write_statistics (:100-115).  On success *out / *out_len is the file image
 * in ctx-owned host memory, valid until the next call on ctx; counts (nqueues
 * uint64) and *n_rows are set.  RSS_CSV_COUNTS_ONLY skips the per-row outputs
 * and the file (out / out_len may be NULL).  Non-canonical input or a body of 4 GiB
 * or more -> RSS_ENOTSUP (take the host or pandas path).
 */
#define RSS_CSV_COUNTS_ONLY 1u
int rss_csv_hash_text(rss_ctx* ctx, const rss_key* key, const char* text, size_t len,
                      uint32_t htable, uint32_t nqueues, const uint32_t* reta, uint32_t flags,
                      const char** out, size_t* out_len, uint64_t* counts, size_t* n_rows);

/*
 * rss_csv_hash_text from file to file: the input streams through two pinned staging
 * buffers of ctx (read of chunk k+1 overlaps the upload of chunk k) and the output
 * rows stream back the same way (download of chunk k+1 overlaps the write of chunk
 * k), so no file-sized host buffer exists.  Bodies of any size are processed in
 * line-aligned segments below 4 GiB (3 GiB; RSS_CSV_SEGMENT_BYTES lowers it), counts
 * summed over the segments and rows written after the last one.  out_path may be NULL with
 * RSS_CSV_COUNTS_ONLY.  An unreadable input or an output that cannot be created is
 * RSS_ENOTSUP as well: the pandas path then raises the reference's error.
 */
int rss_csv_hash_file(rss_ctx* ctx, const rss_key* key, const char* in_path, const char* out_path,
                      uint32_t htable, uint32_t nqueues, const uint32_t* reta, uint32_t flags,
                      uint64_t* counts, size_t* n_rows);

/*
 * The IPv6 `--ipv6 --csv` job on the device, same contracts as rss_csv_hash_text /
 * rss_csv_hash_file: rows are the canonical IPv6 form of rss_csv_parse6 (RFC 4291 text,
 * no embedded IPv4 or zone), hashed with rss_hash6_device (or rss_hash6_device_reta),
 * and each output row is the input row's own text plus ",hash,queue" -- the bytes
 * rss_csv_format6 writes, which are the pandas path's (ingest.py / simulator.py:100-115).
 */
int rss_csv6_hash_text(rss_ctx* ctx, const rss_key6* key, const char* text, size_t len,
                       uint32_t htable, uint32_t nqueues, const uint32_t* reta, uint32_t flags,
                       const char** out, size_t* out_len, uint64_t* counts, size_t* n_rows);
int rss_csv6_hash_file(rss_ctx* ctx, const rss_key6* key, const char* in_path,
                       const char* out_path, uint32_t htable, uint32_t nqueues,
                       const uint32_t* reta, uint32_t flags, uint64_t* counts, size_t* n_rows);

/* rss_key_search_device on host buffers (keys: nkeys prepared keys; h_counts:
 * nkeys x nqueues uint64).  Synchronous. */
int rss_key_search_host(rss_ctx* ctx, const rss_key* keys, size_t nkeys,
                        const rss_tuple4* h_tuples, size_t n, uint32_t htable,
                        uint32_t nqueues, uint64_t* h_counts);

/* rss_hash6_device on host buffers: rss_hash_host's contract and path (the same staging,
 * small-batch path, pipeline and direct DMA of page-locked buffers), 36-byte tuples. */
int rss_hash6_host(rss_ctx* ctx, const rss_key6* key, const rss_tuple6* h_tuples, size_t n,
                   uint32_t htable, uint32_t nqueues, uint32_t* h_hash, uint32_t* h_queue,
                   uint64_t* h_counts, uint32_t flags);

/*
 * ---- pcap input (host) ----
 * One packed 4-tuple per IPv4 packet of a classic libpcap image (either byte
 * order, us/ns timestamps) or a pcapng image (sections of either byte order,
 * per-interface link types, enhanced / simple / obsolete packet blocks; other
 * blocks skipped).  Link types: Ethernet incl. 802.1Q/802.1ad tags, Linux cooked
 * v1, raw IPv4.  TCP/UDP/SCTP packets carry their ports; other protocols and every
 * fragment carry ports 0 (the 2-tuple hash, as NICs do).  protocols (nullable)
 * gets the IP protocol byte per tuple.  Non-IPv4 / malformed packets, and packets
 * of interfaces with other link types, are skipped and counted in *skipped.
 * Returns RSS_ENOTSUP for other images; RSS_EINVAL with *n_out = the needed size
 * when cap is too small.
 */
int rss_pcap_parse(const uint8_t* data, size_t len, rss_tuple4* tuples, uint8_t* protocols,
                   size_t cap, size_t* n_out, size_t* skipped);

/*
 * The same captures, one rss_tuple6 per IPv6 packet (link types as above plus raw
 * IPv6): the fixed header's addresses; the extension-header chain (hop-by-hop,
 * routing, destination options, AH, fragment) is walked to the upper layer, whose
 * ports count for TCP/UDP/SCTP; fragments, ESP and other upper layers carry ports 0.
 * protocols gets the upper-layer protocol.  IPv4 and malformed packets are skipped.
 */
int rss_pcap_parse6(const uint8_t* data, size_t len, rss_tuple6* tuples, uint8_t* protocols,
                    size_t cap, size_t* n_out, size_t* skipped);

int rss_hash_host_reta(rss_ctx* ctx, const rss_key* key, const rss_tuple4* h_tuples, size_t n,
                       uint32_t htable, const uint32_t* reta, uint32_t nqueues, uint32_t* h_hash,
                       uint32_t* h_queue, uint64_t* h_counts, uint32_t flags);

/* The IPv6 counterparts: rss_hash6_device / rss_hash6_host with the bucket -> queue
 * step through reta[htable] (same limits as rss_hash_device_reta). */
int rss_hash6_device_reta(const rss_key6* key, const rss_tuple6* d_tuples, size_t n,
                          uint32_t htable, const uint32_t* reta, uint32_t nqueues,
                          uint32_t* d_hash, void* d_queue, uint64_t* d_counts, uint32_t flags,
                          void* stream);
int rss_hash6_host_reta(rss_ctx* ctx, const rss_key6* key, const rss_tuple6* h_tuples, size_t n,
                        uint32_t htable, const uint32_t* reta, uint32_t nqueues, uint32_t* h_hash,
                        uint32_t* h_queue, uint64_t* h_counts, uint32_t flags);

/*
 * Multi-GPU host batch (replaces the same rows of Simulator.calc_hash /
 * calc_queue_number / write_statistics as rss_hash_host, simulator.py:74-113).  The n
 * tuples are split into nctx contiguous ranges as sharding.shard_range splits a batch over
 * ranks (n / nctx each, the first n % nctx ranges one tuple longer);
 * context i hashes range i on its own device from its own host thread and copies the
 * hash / queue slice straight into the caller's output range (no collective), and the
 * per-queue counts of all ranges are summed on the host -- exact integers, so identical
 * to one device.  Contexts must be distinct (several may share a device).  reta is
 * NULL for the reference's `% nqueues` mapping, else htable queue ids (as
 * rss_hash_host_reta).  Only RSS_FLAG_ACCUMULATE is honoured.  Synchronous.
 */
int rss_hash_host_multi(rss_ctx* const* ctxs, int nctx, const rss_key* key,
                        const rss_tuple4* h_tuples, size_t n, uint32_t htable,
                        const uint32_t* reta, uint32_t nqueues, uint32_t* h_hash,
                        uint32_t* h_queue, uint64_t* h_counts, uint32_t flags);

/* Number of visible gfx950 devices (0 when there is no GPU). */
int rss_device_count(int* out);

/* Thread-local message describing the last failure on this thread ("" if none). */
const char* rss_last_error(void);

/* RSS_ABI_VERSION of the loaded library. */
int rss_abi_version(void);

#ifdef __cplusplus
}
#endif

#endif /* RSS_TOEPLITZ_H */
