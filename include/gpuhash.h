/*
 * gpuhash.h -- C ABI of the MI355X (gfx950) nonce-search engine.
 *
 * Drop-in for the ONE hot path of mohitreddy1996/BitCoin-Miner: the miner's min-hash
 * loop over a Request's inclusive [Lower, Upper].  The reference has no FFI; the
 * boundary is the Go call site that the unimplemented miner loop would occupy:
 *
 *   src/github.com/cmu440/bitcoin/miner/miner.go:15   // TODO: implement this!
 *     spec (p1.pdf pp.12-14): for n in [Lower, Upper] { h := bitcoin.Hash(Data, n) }
 *     keep the least h and its nonce, reply bitcoin.NewResult(h, n)
 *   src/github.com/cmu440/bitcoin/hash.go:11-15        bitcoin.Hash(msg, nonce) uint64
 *   src/github.com/cmu440/bitcoin/message.go:25-42     NewRequest(data, lower, upper),
 *                                                      NewResult(hash, nonce)
 *
 * A Go miner binds it with cgo (INTEGRATION.md shows the stub).  Plain C types only:
 * pointers + sizes + uint64; no torch, no HIP types.  All integers host-endian.
 *
 * Semantics reproduced bit-exactly:
 *   Hash(msg, n) = big-endian uint64 of SHA-256(msg ‖ ' ' ‖ decimal(n))[0:8]
 *   gpuhash_min  = argmin over the INCLUSIVE range of the key (Hash, nonce): the least
 *                  hash, and among equal hashes the lowest nonce (what an ascending
 *                  scan with strict '<' returns).  Overflow-safe at upper = 2^64-1.
 *
 * Threading: calls on one context are serialised internally (a second caller waits);
 * separate contexts run concurrently.  gpuhash_close must not race other calls on
 * the same context.  Every entry point leaves the calling thread's current HIP device
 * as it found it (device work may run on the caller's thread, which a cgo-locked
 * goroutine or a torch process may share).
 *
 * Errors are negative return codes (gpuhash_strerror); nothing is printed, and no C++
 * exception crosses the ABI (allocation failures map to GPUHASH_ENOMEM, any other
 * host-side failure, e.g. thread creation, to GPUHASH_EHIP).  GPUHASH_EINVAL and
 * GPUHASH_ETOOLONG are deterministic argument errors: retrying the same call elsewhere
 * fails the same way.  GPUHASH_ENODEV / EHIP / ENOMEM are device or resource errors.  The HIP
 * path is the only compute path: with no usable device gpuhash_open fails with
 * GPUHASH_ENODEV -- there is no silent CPU fallback.
 */
#ifndef GPUHASH_H
#define GPUHASH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GPUHASH_OK 0
#define GPUHASH_EINVAL (-1)   /* null pointer, lower > upper, bad device list / count */
#define GPUHASH_ENODEV (-2)   /* no usable gfx950 device */
#define GPUHASH_EHIP (-3)     /* a HIP runtime call or kernel launch failed */
#define GPUHASH_ETOOLONG (-4) /* msg_len > GPUHASH_MAX_MSG */
#define GPUHASH_ENOMEM (-5)   /* device or host allocation failed */

/* The reference carries the message in a JSON frame inside <=2000-byte LSP datagrams
 * (lspnet/conn.go:35), so real messages are ~1.3 KB at most; the engine accepts more. */
#define GPUHASH_MAX_MSG (1u << 20)

typedef struct gpuhash_ctx gpuhash_ctx;

/* Per-call measurements of the last gpuhash_min / gpuhash_hash_range on a context. */
typedef struct gpuhash_stats {
    uint64_t nonces;          /* nonces searched by the last call                     */
    uint32_t launches;        /* scan-kernel launches (all devices)                   */
    uint32_t ndevices;        /* devices that received a non-empty shard              */
    double wall_ms;           /* host wall time of the call                           */
    double kernel_ms;         /* sum over devices of HIP-event time of scan launches  */
    double max_dev_kernel_ms; /* slowest device's scan-kernel time                    */
} gpuhash_stats;

/* One scan-kernel launch of the last call (bench.py derives the dominant kernel's
 * average launch time and algorithmic work from these). */
typedef struct gpuhash_launch_record {
    int32_t device;   /* HIP ordinal of the context entry that ran the launch       */
    int32_t J;        /* kernel variant: loop-word index in the final block (0..15) */
    int32_t C2;       /* 1: lane digits spill into block B-1, per-nonce schedule;   */
                      /* 2: block B's W_0/W_1 hold only loop digits, schedules      */
                      /*    shared per wave through LDS; 3: lane table (per-lane    */
                      /*    block-B schedule, block B-1 state from a p-table)       */
    int32_t EX;       /* 1: extra all-constant padding block                        */
    int32_t digits;   /* decimal digits of every nonce in the launch                */
    int32_t c;        /* 64-byte blocks holding nonce digits (1 or 2)               */
    int32_t shard;    /* index of the context entry (gpuhash_open's list position)  */
    int32_t stream_device; /* ordinal the HIP runtime reports for the stream the    */
                      /*    kernel was launched on (hipStreamGetDevice): evidence   */
                      /*    that the shard ran on `device`, not on device 0         */
    uint64_t lo, hi;  /* the shard's inclusive nonce range in this slice            */
    uint64_t nonces;  /* nonces covered by the launch                               */
    double ms;        /* HIP-event time of the launch on the device's stream        */
    double sclk_mhz;  /* shader clock over the launch, measured in the kernel:      */
                      /*    s_memtime ticks / s_memrealtime (100 MHz) of workgroup 0 */
} gpuhash_launch_record;

/* Opens the listed devices (HIP ordinals); ndevices == 0 means every visible device.
 * Allocates per-device streams, events and a small candidate buffer.  An ordinal may be
 * listed more than once (each entry is a separate shard with its own stream).
 * Replaces: nothing in the reference (the miner would call it once at start-up,
 * miner.go:8-16). */
int gpuhash_open(const int *devices, int ndevices, gpuhash_ctx **out);

/* Number of devices a context drives. */
int gpuhash_ndevices(const gpuhash_ctx *ctx);

/* Number of visible HIP devices (0 if none).  Lets a host check a device list before
 * gpuhash_open (bench.py --gpus N refuses N above it).  Replaces nothing in the reference. */
int gpuhash_device_count(void);

/* The static partition gpuhash_min applies over n devices, for hosts that shard one
 * search over PROCESSES instead (gpuhash.dist: one process per GPU):
 * nshards contiguous shards of the inclusive [lower, upper], in order, of equal estimated
 * cost -- nonces x the layout's relative cost per digit group, so a range whose digit
 * groups differ in SHA blocks (message lengths 45-54, 1 -> 2 blocks at some digit count)
 * is balanced by work, not by count.  Shard k is [out_lower[k], out_upper[k]];
 * out_lower[k] > out_upper[k] (1 > 0) marks an empty shard.  Returns the number of
 * non-empty shards, or GPUHASH_EINVAL (nshards < 1, null outputs, lower > upper) /
 * GPUHASH_ETOOLONG.  Host-only: needs no device.  Replaces the server's job split of
 * p1.pdf p.14 within one node; the merge is the same (hash, nonce) argmin. */
int gpuhash_shard_range(size_t msg_len, uint64_t lower, uint64_t upper, int nshards,
                        uint64_t *out_lower, uint64_t *out_upper);

/* gpuhash_shard_range under a layout policy (gpuhash_set_layout_policy's values): the
 * cost of a digit group depends on the layout that runs it, so gpuhash_min's in-process
 * cuts under a non-AUTO policy are these, and a host sharding over processes with that
 * policy passes it here to cut the same way.  gpuhash_shard_range is this with
 * GPUHASH_LAYOUT_AUTO.  GPUHASH_EINVAL also for an invalid policy.  Host-only. */
int gpuhash_shard_range_policy(size_t msg_len, uint64_t lower, uint64_t upper, int nshards, int policy,
                               uint64_t *out_lower, uint64_t *out_upper);

/* Layout choice for a digit group whose digits straddle two SHA blocks with the loop word
 * at W_1 of the last block, i.e. 5-8 digits in the last block.  Let
 * q = the digits in block B's W_0/W_1 (RQ = 10^q nonces per block B-1 value), nb1 = the
 * digits in block B-1, span = the search's nonces in that digit group, and N =
 * (span - 1) / RQ + 2, the block B-1 values such a span can touch.  This comment is
 * the ONE statement of the rule; csrc/plan.cpp (layout_for) implements it and
 * tests/test_plan.py checks the two against each other.
 *   AUTO (default)  span < 2 * RQ                                -> C2 = 1 (classic)
 *                   else nb1 >= 3 and N > GPUHASH_LANETABLE_MAX  -> C2 = 2 (two-word loop)
 *                   else                                         -> C2 = 3 (lane table)
 *   UNIFORM         nb1 >= 3 -> C2 = 2, else C2 = 3
 *   CLASSIC         C2 = 1 always (the per-nonce-schedule layout)
 *   LANETABLE       C2 = 3 up to N = GPUHASH_LANETABLE_MAX, C2 = 2 beyond it (each value
 *                   costs 64 B of table and one compression, so the cap bounds memory)
 * Results are identical under every policy; only speed differs.  Exposed for tuning and
 * so that parity tests can drive every kernel over small ranges.  Replaces nothing in
 * the reference. */
#define GPUHASH_LAYOUT_AUTO 0
#define GPUHASH_LAYOUT_UNIFORM 1
#define GPUHASH_LAYOUT_CLASSIC 2
#define GPUHASH_LAYOUT_LANETABLE 3
#define GPUHASH_LANETABLE_MAX 65536u
/* Tail-digit launches, for any policy above: a digit group whose last
 * digit-bearing word holds ONE digit after a word of four (e.g. "bradfitz" at 8 and 12
 * digits) would loop over only 10 values per 256-lane row; it runs instead as ten
 * launches, one per last digit t, over the nonces = t (mod 10) with t a constant message
 * byte, looping over the previous word's 10^4 values.  Taken when the search spans at
 * least GPUHASH_TAIL_MIN_SPAN nonces of the group (below that, the launches' partial rows
 * cost more than the short loop); OR GPUHASH_LAYOUT_TAIL_ALWAYS or _NEVER into the policy
 * to force either way (parity tests, tuning).  Results are identical either way. */
#define GPUHASH_LAYOUT_TAIL_ALWAYS 16
#define GPUHASH_LAYOUT_TAIL_NEVER 32
#define GPUHASH_TAIL_MIN_SPAN 8589934592ull
int gpuhash_set_layout_policy(gpuhash_ctx *ctx, int policy);

/* argmin_{n in [lower, upper]} (Hash(msg, n), n) -> *out_hash, *out_nonce.
 * Replaces the miner loop of p1.pdf pp.12-14 (miner.go:15) and feeds
 * bitcoin.NewResult(hash, nonce) (message.go:36-42).  msg is read during the call
 * only (cgo pointer rules); the range is split statically over the context's devices
 * (one host thread + one stream each), reduced on the host.  Blocking.  Any span is
 * accepted, up to the full [0, 2^64-1]: spans over 2^38 nonces per device run as
 * consecutive slices (env GPUHASH_SLICE_NONCES overrides the per-device slice). */
int gpuhash_min(gpuhash_ctx *ctx, const uint8_t *msg, size_t msg_len, uint64_t lower,
                uint64_t upper, uint64_t *out_hash, uint64_t *out_nonce);

/* Same search, caller-chosen work-item granularity (r values per workgroup; 0 =
 * default).  Exposed for tuning and for parity tests of the chunked paths. */
int gpuhash_min_ex(gpuhash_ctx *ctx, const uint8_t *msg, size_t msg_len, uint64_t lower,
                   uint64_t upper, uint32_t rchunk, uint64_t *out_hash, uint64_t *out_nonce);

/* out[i] = Hash(msg, lower + i) for i < count, computed on the first device by the
 * SAME kernels as gpuhash_min (per-nonce dump mode).  count <= 2^26; lower + count - 1
 * must not wrap.  Parity/diagnostic API (batch form of hash.go:11-15). */
int gpuhash_hash_range(gpuhash_ctx *ctx, const uint8_t *msg, size_t msg_len,
                       uint64_t lower, uint64_t count, uint64_t *out);

/* bitcoin.Hash(msg, nonce) for ONE nonce on the host (hash.go:11-15): the miner's
 * optional self-check of a returned (hash, nonce); never used by gpuhash_min. */
uint64_t gpuhash_hash_cpu(const uint8_t *msg, size_t msg_len, uint64_t nonce);

/* Measurements of the last call on ctx. */
int gpuhash_last_stats(const gpuhash_ctx *ctx, gpuhash_stats *out);

/* Copies up to cap launch records of the last call; returns how many exist. */
int gpuhash_last_launches(const gpuhash_ctx *ctx, gpuhash_launch_record *out, int cap);

void gpuhash_close(gpuhash_ctx *ctx);

const char *gpuhash_strerror(int rc);

/* Library/ABI version, "gpuhash <major>.<minor> gfx950 build=<id>": <id> is a hash of
 * the sources the library was built from (bench.py matches it against profiled builds). */
const char *gpuhash_version(void);

#ifdef __cplusplus
}
#endif

#endif /* GPUHASH_H */
