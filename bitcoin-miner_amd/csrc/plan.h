// plan.h -- nonce-range planner shared by the HIP host library and the CPU self-check.
//
// The reference computes bitcoin.Hash(msg, n) = BE64(SHA256(msg ‖ ' ' ‖ dec(n))[0:8])
// (src/github.com/cmu440/bitcoin/hash.go:11-15) for every n of the miner's inclusive
// [Lower, Upper] (bitcoin/message.go:25-32, loop spec'd in p1.pdf pp.12-14) and keeps
// the least.  The planner turns one such search into launches whose SHA-256 message
// layout is FIXED per launch, so the kernels can precompute everything that does not
// depend on the nonce:
//
//   digit group   all nonces of one decimal length d (1..20): L = m+1+d hashed bytes
//   launch        nonces H·10^(s+q) + p·10^q + r sharing the h = d-s-q leading digits H
//     loop digits r: the q (1..4) digits that sit in the LAST digit-bearing 32-bit word
//                    W_J of the final block B -> the only per-nonce message word
//     lane digits p: the s (0..8) digits just before word J, i.e. virtual words J-1 and
//                    J-2 (these may fall into block B-1: "C2" layouts)
//     (C2 = 2, J = 1: the loop takes the 4 digits of W_0 as well -- q = 4 + digits of
//      W_1, up to 8 -- so block B holds loop digits only and its schedule is uniform;
//      the lanes then take only digits of block B-1)
//     (C2 = 3, J = 1, "lane table": the roles swap -- each LANE takes one value of the
//      q = 4 + q1 digits of block B's W_0/W_1 and keeps that block's whole K+W schedule
//      in registers, built once per row; the LOOP runs over the s digits at the end of
//      block B-1, whose chaining values the host precomputes (16 words per value, the
//      launch's "p-table").  For straddles whose block B-1 holds too few digits to fill
//      C2 = 2's 256-lane rows, e.g. message lengths = 61, 62 mod 64 at 6-10 digits)
//     uniform     : prefix bytes, H's digits, 0x80, zero pad, bit length -> host
//                    precomputes the midstate, the uniform words and the rounds that
//                    only read uniform words
//   tail digit    (plain layouts whose last digit-bearing word holds ONE digit: a loop of
//                  only 10 values per row, whose per-row setup then costs ~2.6%) the last
//                  digit t is fixed per launch: ten launches, one per t, each searching the
//                  nonces = t (mod 10) as k = nonce / 10 with t a constant message byte, so
//                  the loop word is the previous, 4-digit word (R = 10^4)
//   work item     (a group of 256 consecutive lane values p) × (a chunk of r values)
//                 = one workgroup of the kernel
//
// Kernel variant = (J, C2, EX): J = index of the loop word in block B (0..15);
// C2 = lane digits spill into block B-1, which is then compressed per lane; EX = the
// 0x80/length need an extra all-constant block B+1 (last digit at byte >= 55 of B).
#pragma once
#include <stdint.h>

#include <vector>

#include "gpuhash.h"  // GPUHASH_LANETABLE_MAX: the layout-policy rule is stated there

namespace gpuhash {

static constexpr uint32_t kIV[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                                    0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};

extern const uint32_t kK[64];

// Per-launch constants, passed by value as the kernel argument (lives in SGPRs/
// the kernarg segment; never touches HBM in the hot loop).  Keep POD + 4-byte words.
struct LaunchDesc {
    uint32_t U[16];    // block B words with every lane/loop digit byte zeroed
    uint32_t S0[8];    // non-C2: block-B state after the uniform rounds 0..J-3
    uint32_t CV[8];    // non-C2: chaining value entering block B
    uint32_t U1[16];   // C2: block B-1 words, lane digit bytes zeroed
    uint32_t S1[8];    // C2: block B-1 state after its uniform rounds 0..13
    uint32_t CV1[8];   // C2: chaining value entering block B-1
    uint32_t KWX[64];  // EX: K[t] + W[t] of the all-constant block B+1
    uint32_t mask_lo;  // bytes of virtual word J-1 that take ascii4(p % 10^4)
    uint32_t mask_hi;  // bytes of virtual word J-2 that take ascii4(p / 10^4)
    uint32_t qmask;    // low q bytes
    uint32_t loop_shift;  // bit position of the last loop digit's byte in W_J
    uint32_t R;        // 10^q  (r in [0, R))
    uint32_t rchunk;   // r values per work item
    uint32_t nrchunks; // ceil(R / rchunk)
    uint32_t p_first, p_last;  // lane values covered by this launch
    uint32_t r_first, r_last;  // r bounds at p_first / p_last (edges of [lo, hi])
    // C2 with J == 0: every word of block B is wave-uniform (the lanes only vary block
    // B-1), so its whole schedule K[t] + W_t(r) is a per-r table, built once per digit
    // group by k_ktab; the scan reads row r at ktab + tab_off + 64*r (scalar loads).
    uint32_t tab_off;
    // C2 = 3: tab_off = word offset of this launch's p-table (16 words per loop value:
    // block B-1's chaining value, then round 0's per-row sums inv0 and t20 of block B)
    uint32_t R1;       // C2 = 2, 3: 10^(digits of W_1); (W_0, W_1) digits = (x / R1, x % R1)
    uint32_t RQ;       // C2 = 3: 10^q, lane values per loop value
    uint64_t base;     // nonce = base + p·R + r  (C2 = 3: base + r·RQ + p, p = lane value)
    uint32_t lt_p0;    // C2 = 3: block B-1 value of loop value 0 (p-table entry k: lt_p0 + k)
    // tail-digit launches (below): the kernel's k = base + p·R + r is the nonce without its
    // last digit, nonce = k·stride + tail; plain launches: stride 1, tail 0
    uint32_t stride;
    uint32_t tail;
    uint32_t pad2_;
};

struct Launch {
    int J;          // loop word index in block B
    int C2;         // 1: lane block B-1 compressed per lane; 2: and W_0, W_1 are loop words
    int EX;         // extra constant padding block
    int d, q, s;    // digits, loop digits, lane digits
    int c;          // 64-byte blocks that hold nonce digits (the SURVEY 8(d) "c")
    uint64_t lo, hi;      // first and last nonce covered (every stride-th nonce from lo)
    uint32_t stride = 1;  // 10 for a tail-digit launch: the nonces = tail (mod 10) in [lo, hi]
    uint32_t nblocks;     // grid size (workgroups of 256)
    LaunchDesc desc;
    uint32_t nptab = 0;          // C2 = 3: p-table words (16 per loop value, LaunchDesc::tab_off)
    std::vector<uint32_t> ptab;  // C2 = 3: the p-table, filled on the host only when planned
                                 //   with host_ptab (the CPU replay); the library builds it
                                 //   on the device (k_ptab)
};

// Largest number of lane digits; 10^kMaxLane lanes per launch.
static constexpr int kMaxLane = 8;
static constexpr int kBlock = 256;
static constexpr int kMaxLaunchDigits = 10;   // s + q <= 10  -> <= 10^10 nonces per launch
// C2 = 2 launches: s + q <= 12 still keeps rows * R = ceil(10^s / 256) * 10^q < 2^32
static constexpr int kMaxLaunchDigitsU2 = 12;

// Choice between the J = 1 straddling layouts (plan.cpp layout_for); the rule is stated
// once, in include/gpuhash.h above GPUHASH_LAYOUT_AUTO.
enum LayoutPolicy { kLayoutAuto = 0, kLayoutUniform = 1, kLayoutClassic = 2, kLayoutLaneTable = 3 };
// policy flags for the tail-digit layouts (include/gpuhash.h): taken for digit groups the
// search spans kTailMinSpan nonces of, or always / never with the flags
static constexpr int kLayoutMask = 15;
static constexpr int kLayoutTailAlways = GPUHASH_LAYOUT_TAIL_ALWAYS;
static constexpr int kLayoutTailNever = GPUHASH_LAYOUT_TAIL_NEVER;
static constexpr uint64_t kTailMinSpan = GPUHASH_TAIL_MIN_SPAN;
// C2 = 3: at most this many loop values (p-table entries) per launch, and AUTO / LANETABLE
// take the layout only for searches touching at most kMaxLtTable block B-1 values (4 MB)
static constexpr uint32_t kMaxLtLoop = 1024;
static constexpr uint64_t kMaxLtTable = GPUHASH_LANETABLE_MAX;

// Plans [lower, upper] (inclusive, lower <= upper) of `msg`.  `rchunk_max` caps the r
// values per work item (0 = default).  Appends to `out`.
void plan_range(const uint8_t* msg, uint64_t len, uint64_t lower, uint64_t upper,
                std::vector<Launch>& out, uint32_t rchunk_max = 0, int policy = kLayoutAuto,
                bool host_ptab = false);

struct Shard {
    uint64_t lo, hi;  // inclusive
    int empty;        // 1 when the range has fewer nonces than shards
};

// Splits [lower, upper] into n contiguous shards of about equal estimated cost
// (nonce count weighted by the layout's per-nonce cost).  Used to spread one search
// over the devices of a context (static contiguous shards).
// `policy` = the layout policy the shards will be planned with (plan_range).
std::vector<Shard> shard_range(uint64_t msg_len, uint64_t lower, uint64_t upper, int n,
                               int policy = kLayoutAuto);

// Relative per-nonce cost of digit group d for a message of msg_len bytes, when a call
// covers `span` of its nonces (0 = the whole group) under layout policy `policy`.
double group_cost(uint64_t msg_len, int d, uint64_t span = 0, int policy = kLayoutAuto);

// The same cost model summed over a plan's launches (nonces x their layout's cost).
double plan_cost(const std::vector<Launch>& plan);

// Host SHA-256 pieces used for midstates (not a hashing path of its own).
void sha256_compress(uint32_t st[8], const uint32_t w16[16]);
void sha256_rounds(uint32_t st[8], const uint32_t w[64], int t_begin, int t_end);
void sha256_expand(uint32_t w[64]);
uint64_t hash_host(const uint8_t* msg, uint64_t len, uint64_t nonce);

int num_digits(uint64_t n);
uint64_t pow10u(int k);
uint32_t ascii4(uint32_t x);  // x < 10^4 -> 4 ASCII digits, big-endian in a word

}  // namespace gpuhash
