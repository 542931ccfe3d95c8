// superkmer.h -- minimizers of k-mers, 21 <= k <= 32 (the super-k-mer count of count_sk2.h,
// the graph phase's bucketed lookups, the sharded path's owners).
//
// The minimizer of a k-mer -- the smallest hash over its w = k - m + 1 canonical m-mers -- is
// also the minimizer of its twin (both hold the same canonical m-mers), so partitioning k-mers
// by minimizer puts every occurrence of a canonical k-mer into one bucket, and consecutive
// windows of a read that share their minimizer (a super-k-mer, ~(w + 1) / 2 windows on random
// sequence) travel as one record (count_sk2.h).  SolidIndex (graph.h, sk = 1): a key's bucket
// = top bits of its minimizer, first probe slot sk_slot(key).
#pragma once
#include "count_part.h"

namespace ec {

constexpr int SK_M = 15;                        // minimizer length (canonical m-mers, odd: no palindromes)
constexpr int SK_MIN_K = 21;                    // super-k-mer mode for SK_MIN_K <= k <= 32
constexpr int SK_W_MAX = 32 - SK_M + 1;         // windows per m-mer block (w) at k = 32

struct MinCfg {
    int k, m, w;
    uint32_t mmask;  // 2m bits
    int msh;         // 2m - 2
};

inline MinCfg sk_cfg(int k) {
    MinCfg c;
    c.k = k;
    c.m = SK_M;
    c.w = k - SK_M + 1;
    c.mmask = (1u << (2 * SK_M)) - 1;
    c.msh = 2 * SK_M - 2;
    return c;
}

// m-mer order: a bijective 32-bit mix of the canonical code (equal hashes = equal m-mers).
// One multiply: the minimizer density it gives on random sequence (0.1119 at w = 17) matches
// a random order's 2 / (w + 1) as closely as murmur's three-multiply finaliser (0.1112), and
// the bucket bits come from min_remix.
__host__ __device__ inline uint32_t mmer_hash(uint32_t x) {
    x *= 0x9E3779B1u;
    return x ^ (x >> 15);
}

// the minimizer's identity as used downstream: the minimum hash rotated so that its LOW 14
// bits are the top ones -- the minimum of w hashes crowds its high bits towards 0, its low bits
// stay uniform -- so the fine bin, coarse and final bucket (top bits) and the owner ranges are
// even.  Bijective; k_skpart_w takes the bucket bits as runv << 18 (no remix per run).
__host__ __device__ inline uint32_t min_remix(uint32_t x) { return (x >> 14) | (x << 18); }
// the same for placements that use up to ~20 bucket bits (count_wide.h minimizer buckets: 14
// fine + up to 6 third-level bits, join_w.h junction buckets): min_remix's bits after the top 14
// are the minimum's HIGH bits -- almost always 0 (the minimum of w ~ 37 hashes is ~2^32 / 38) --
// so they put every key of a fine bucket into its first sub-bucket.  Here the top 20 bits are
// the minimum's low 20 bits, uniform
__host__ __device__ inline uint32_t min_remix_w(uint32_t x) { return (x >> 20) | (x << 12); }

__host__ __device__ inline uint32_t rev2_32(uint32_t x) {
    x = ((x >> 2) & 0x33333333u) | ((x & 0x33333333u) << 2);
    x = ((x >> 4) & 0x0F0F0F0Fu) | ((x & 0x0F0F0F0Fu) << 4);
    return (x >> 24) | ((x >> 8) & 0xFF00u) | ((x << 8) & 0xFF0000u) | (x << 24);
}

// hash of the canonical form of forward m-mer f
__host__ __device__ inline uint32_t mmer_canon_hash(uint32_t f, const MinCfg &g) {
    const uint32_t r = rev2_32(f ^ g.mmask) >> (32 - 2 * g.m);
    return mmer_hash(f < r ? f : r);
}

// minimizer of k-mer code c (the graph phase's bucket of a key, the sharded path's owner):
// the twin's m-mer at offset p is the reverse complement of c's m-mer p, so one 64-bit
// reversal replaces a 32-bit one per m-mer (= mmer_canon_hash of every m-mer)
__host__ __device__ inline uint32_t minimizer_of(uint64_t c, const MinCfg &g) {
    const uint64_t tc = twin64(c, g.k);
    uint32_t v = 0xFFFFFFFFu;
    for (int p = 0; p < g.w; p++) {
        const uint32_t f = (uint32_t)(c >> (2 * (g.k - g.m - p))) & g.mmask;
        const uint32_t r = (uint32_t)(tc >> (2 * p)) & g.mmask;
        const uint32_t h = mmer_hash(f < r ? f : r);
        v = h < v ? h : v;
    }
    return min_remix(v);
}

// final bucket of a minimizer (bbits <= FINE_BITS)
__host__ __device__ inline unsigned int sk_bucket_of(uint32_t v, int bbits) { return bbits ? v >> (32 - bbits) : 0u; }

// first probe slot of canonical key c in a super-k-mer bucket table (top bits used)
__host__ __device__ inline unsigned int sk_slot(unsigned long long c) {
    return (unsigned int)c * 0x9E3779B1u + (unsigned int)(c >> 32) * 0x85EBCA77u;
}

}  // namespace ec
