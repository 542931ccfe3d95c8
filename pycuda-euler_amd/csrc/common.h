// common.h -- shared device/host helpers for libeulerhip (gfx950 / CDNA4, wave64).
#pragma once
#include <cstring>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string>

#include "../../include/eulerhip.h"

namespace ec {

constexpr uint32_t NONE32 = 0xFFFFFFFFu;
constexpr uint64_t NONE64 = ~0ull;
constexpr uint64_t EMPTY_KEY = ~0ull;  // canonical 2-bit keys (k <= 32) never equal all-ones

// thread-local last error (ec_last_error)
void set_error(const char *fmt, ...);

// Test / diagnostic overrides.  Read once per C-ABI call (refresh_knobs) and only when
// EULERHIP_DEBUG is set: without it the library's behaviour never depends on the environment.
// Each forces a path the default heuristics would not take on small inputs, so the oracle can
// check it (tests/conftest.py sets EULERHIP_DEBUG=1).
struct Knobs {
    bool no_sk2 = false;        // EULERHIP_NO_SK2: no super-k-mer records (count_sk2.h)
    bool no_v2 = false;         // EULERHIP_NO_V2: no fixed-capacity runs (count_v2.h)
    bool force_filter = false;  // EULERHIP_FORCE_FILTER: seen-twice filter buckets at any size
    bool no_filter = false;     // EULERHIP_NO_FILTER
    int filter_pmax = 0;        // EULERHIP_FILTER_PMAX: part tables 2^pmax (0 = from the estimate)
    int filter_pmin = -1;       // EULERHIP_FILTER_PMIN
    float part_keys = 0.0f;     // EULERHIP_PART_KEYS: keys per part table (0 = PART_KEYS)
    int v2_r10 = -1;            // EULERHIP_V2_R10: 10-B window records 1 = forced, 0 = never
    int refine_rs = 0;          // EULERHIP_REFINE_RS: refine slices per coarse bucket (0 = 8)
    int rank_sync = 0;          // EULERHIP_RANK_SYNC=1: tile ranking with host-read counts (A/B)
    int rj_div = 0;             // EULERHIP_RJ_DIV: rank_supers_async's Wyllie grids cover N / RJ_DIV rulers (A/B)
    int tile_plan = -1;         // EULERHIP_TILE_PLAN=0: fixed rank tiles, not cut at bucket starts (A/B)
    int no_spec = 0;            // EULERHIP_NO_SPEC=1: no speculative refine launch (count_sk2, A/B)
    bool merge_mix = false;     // EULERHIP_MERGE_MIX: key-hash buckets / owners instead of minimizers
    int skf_merge = 1;          // EULERHIP_SKF_MERGE: error-rich records merged before the filter (0 off, 2 2560-entry tables)
    bool merge_decode = false;  // EULERHIP_MERGE_DECODE: the owner merge reads a decoded copy of the received records
    int wide_runs = 1;          // EULERHIP_WIDE_RUNS: 128-bit keys on minimizer buckets partition runs (0: windows, 2: runs expanded to windows)
    bool wide_general = false;  // EULERHIP_WIDE_GENERAL: k > 32 on the HBM table
    int wide_max_bbits = -1;    // EULERHIP_WIDE_MAX_BBITS: cap the wide buckets (forces overflow)
    int wide_l3 = 0;            // EULERHIP_WIDE_L3: third partition level of 2^n sub-buckets at any size
    long long wide_l3_cap = 0;  // EULERHIP_WIDE_L3_CAP: its sub-bucket capacity (forces its overflow)
    int join_links = -1;        // EULERHIP_JOIN_LINKS: links by the half-edge join 1 = always, 0 = never
    int junction_bt = -1;       // EULERHIP_JUNCTION_BT: most join bucket bits of the junction join (<= 14)
    int junction_sb = 0;        // EULERHIP_JUNCTION_SB: at least this many sub-bucket bits
    int junction_claim = 0;     // EULERHIP_JUNCTION_CLAIM: slots a join table may claim (forces overflows)
    int no_char_pack = 0;
    int wr_one = 0;             // EULERHIP_WR_ONE: k_bucket_wr as one 1024-thread workgroup per CU (round 5)       // EULERHIP_NO_CHAR_PACK: contig characters to host as ASCII
    int sk2_elim = 0;           // EULERHIP_SK2_ELIM: entries a k_skpart_w wave may buffer (>= 128)
    int join_cap = 0;           // EULERHIP_JOIN_CAP: its level regions' capacity (forces the fallback)
    int host_chunks = 0;        // EULERHIP_HOST_CHUNKS: host-input chunks (0 = ~32 MiB each)
    bool sk2_stats = false;     // EULERHIP_SK2_STATS: k_skbucket dedup statistics on stderr
    int sk2_claim = 0;          // EULERHIP_SK2_CLAIM: k_skbucket3 record-table claim cap (tests: overflow list)
    bool no_skb3 = false;       // EULERHIP_NO_SKB3: k_skbucket's 8192-bucket plan instead of k_skbucket3 (A/B)
    bool no_slot_groups = false; // EULERHIP_NO_SLOT_GROUPS: k_skpart_w read groups not rounded to resident slots (A/B)
    bool verbose = false;       // EULERHIP_VERBOSE: count-path fallbacks on stderr
    int rank = -1;              // EULERHIP_RANK: list ranking 0 = tile contraction (rank_tile.h), 1 = node ruling set
    int sk_filt = -1;           // EULERHIP_SK_FILT: 0 = error-rich inputs on window records, not k_skbucket_filt
    int skf_keys = 0;           // EULERHIP_SKF_KEYS: k_skbucket_filt's keys-per-table cap (forces its overflow)
    int wide_mb = -1;        // EULERHIP_WIDE_MB=0: 128-bit keys bucketed by mix128, not by minimizer
    int sruler_mask = 0;     // EULERHIP_SRULER_MASK: first ruler pass of the super list takes 1 / (mask + 1)
    int join_local = -1;
    int junction_radix = -1;
    int jl_fcap = -1;        // EULERHIP_JL_FCAP: the local join's foreign-record capacity (tests: overflow)
    int jl_bits_delta = 0;   // EULERHIP_JL_BITS_DELTA: join tables finer / coarser than the count's (tests)
    int upsweep_staged = -1;  // EULERHIP_UPSWEEP_STAGED=1: runs counted by the staged upsweep (A/B)
    int run_packed = -1;      // EULERHIP_RUN_PACKED=0: config 5's run codes gathered from the ASCII reads
    int copy_streams = -1;    // EULERHIP_COPY_STREAMS=2: host-input chunks alternate over two copy streams  // EULERHIP_JUNCTION_RADIX=1: junction buckets by the radix sort at any size     // EULERHIP_JOIN_LOCAL=0: links of minimizer-table ids by the global half-edge join
    int join_mb = -1;        // EULERHIP_JOIN_MB=0: junctions of minimizer-bucketed keys bucketed by mix128
    bool no_small_starts = false; // EULERHIP_NO_SMALL_STARTS: short lists on the general launches (k_starts_small, k_links_small off)
};
void refresh_knobs();
const Knobs &kn();

#define EC_HIP(call)                                                                       \
    do {                                                                                   \
        hipError_t e_ = (call);                                                            \
        if (e_ != hipSuccess) {                                                            \
            ::ec::set_error("%s:%d %s -> %s", __FILE__, __LINE__, #call, hipGetErrorString(e_)); \
            return EC_ERR_HIP;                                                             \
        }                                                                                  \
    } while (0)

#define EC_CHECK(call)                 \
    do {                               \
        int rc_ = (call);              \
        if (rc_ != EC_OK) return rc_;  \
    } while (0)

// ---- 2-bit k-mer algebra (A=0 C=1 G=2 T=3, first base most significant) ------------------
// matches referenceAssembler.py kmers/twin/fw/bw (:7-22) and the reference GPU encoding
// (src/pyencode.py:40 codeF, :62-69 MSB-first packing).
__host__ __device__ inline uint64_t kmask64(int k) { return k >= 32 ? ~0ull : ((1ull << (2 * k)) - 1); }

__host__ __device__ inline uint64_t rev2_64(uint64_t x) {
    x = ((x >> 2) & 0x3333333333333333ull) | ((x & 0x3333333333333333ull) << 2);
    x = ((x >> 4) & 0x0F0F0F0F0F0F0F0Full) | ((x & 0x0F0F0F0F0F0F0F0Full) << 4);
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_bswap64(x);
#else
    return __builtin_bswap64(x);
#endif
}

// reverse complement of a k-mer code (twin, referenceAssembler.py:7-10)
__host__ __device__ inline uint64_t twin64(uint64_t x, int k) { return rev2_64(x ^ kmask64(k)) >> (64 - 2 * k); }

// 64-bit placement hash (xorshift-multiply-xorshift): table placement only, never part of a
// result.  One 64-bit multiply instead of murmur3 fmix64's two: the counting passes hash every
// window and are VALU-bound (measured: k_upsweep 1.59 -> 1.49 ms, k=51 step 42.5 -> 41.5 ms).
// The top bits (buckets, owners, HLL) come from the product's high half, the low bits (slots)
// from its low half xor the high half.
__host__ __device__ inline uint64_t mix64(uint64_t x) {
    x ^= x >> 29;
    x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 32;
    return x;
}

// Bijective placement hash of an n-bit key (n = 2k <= 64): xorshift, multiply mod 2^n, xorshift
// (s = ceil(n/2), so one xorshift step inverts itself).  Its top bits pick the bucket of a key
// and the remaining bits identify the key inside the bucket (count_v2.h 10-byte records), so
// bij_inv recovers the key from (bucket, remnant).
constexpr uint64_t BIJ_C = 0xbf58476d1ce4e5b9ull;
constexpr uint64_t BIJ_CINV = 0x96de1b173f119089ull;  // BIJ_C^-1 mod 2^64
__host__ __device__ inline uint64_t bij_fwd(uint64_t x, int s, uint64_t m) {
    x ^= x >> s;
    x = (x * BIJ_C) & m;
    return x ^ (x >> s);
}
__host__ __device__ inline uint64_t bij_inv(uint64_t x, int s, uint64_t m) {
    x ^= x >> s;
    x = (x * BIJ_CINV) & m;
    return x ^ (x >> s);
}

// ASCII -> 2-bit code; 4 = 'N' (segment break, referenceAssembler.py:29), 5 = invalid byte
__device__ inline uint32_t base_code(uint32_t c) {
    // A=65 C=67 G=71 T=84 N=78
    switch (c) {
    case 'A': return 0;
    case 'C': return 1;
    case 'G': return 2;
    case 'T': return 3;
    case 'N': return 4;
    default: return 5;
    }
}

// Wave-aggregated append: every lane of the wave must call it (convergent).  Lanes with
// pred get consecutive slots of *counter; one atomic per wave instead of one per lane.
__device__ inline unsigned int wave_append(unsigned int *counter, bool pred) {
    const unsigned long long m = __ballot(pred);
    if (!m) return 0;
    const unsigned int lane = threadIdx.x & 63;
    const int leader = __ffsll((long long)m) - 1;
    unsigned int base = 0;
    if ((int)lane == leader) base = atomicAdd(counter, (unsigned int)__popcll(m));
    base = __shfl(base, leader);
    return base + (unsigned int)__popcll(m & ((1ull << lane) - 1));
}

inline unsigned grid_for(uint64_t n, unsigned block, unsigned cap = 1u << 20) {
    uint64_t g = (n + block - 1) / block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (unsigned)g;
}

}  // namespace ec
