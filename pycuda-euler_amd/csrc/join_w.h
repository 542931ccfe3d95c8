// join_w.h -- successor links of 128-bit keys (32 < k <= 63) by a (k-1)-mer half-edge join.
//
// get_contig_forward (referenceAssembler.py:59-73): oriented x -> y iff |fw(x) in d| = 1 (= y),
// |bw(y) in d| = 1 and y != twin(x).  k_neighbors answers it with 8 hash probes per canonical
// key; at config 5's 2e8 keys those are 1.6e9 random sub-table probes (67 ms of a 222 ms step).
// Here the same relation comes out of a bucketed join, every pass sequential:
//
// For an oriented (k-1)-mer o let A(o) = {oriented k-mers in d whose suffix is o} and
// B(o) = {oriented k-mers whose prefix is o}; for x in A(o): fw(x) in d = B(o), and for y in
// B(o): bw(y) in d = A(o).  So x -> y iff A(o) = {x}, B(o) = {y} and y != twin(x).  Twin
// symmetry: A(twin o) = twin(B(o)), B(twin o) = twin(A(o)), so one group per canonical (k-1)-mer
// o^ holds both, and a link x -> y found there also gives twin(y) -> twin(x).
//
//   k_half_emit_l1  per canonical key c (node 2u, twin node 2u+1): two records -- c's suffix s
//                (s < twin s: (s, A, c); else (twin s, B, twin c)) and prefix p (p < twin p:
//                (p, B, c); else (twin p, A, twin c)); a palindromic (k-1)-mer is both its own
//                twin and canonical, so it gets both records -- sorted in LDS straight into the
//                first level's fixed-capacity regions by the top bits of the junction's hash
//   k_refine     1-2 more levels of <= 256-way LDS bucket sorts (the count's refine kernel, fcap
//                mode)
//   k_half_join  per final bucket: an LDS table keyed by o^ collects the distinct node ids of
//                each side (a second distinct id marks the side "many"); every group with one
//                id on each side and y != twin(x) writes succ[x] = y and succ[twin y] = twin x
//
// Record traffic: 2U records of 24 B written once and read + written once per level, then read
// by the join: ~(2 + 2 L) * 48 B per key instead of 8 random probes.  A region or table past
// its capacity makes the caller fall back to k_neighbors / k_succ (same result).
#pragma once
#include "count_wide.h"
#include "graph.h"

namespace ec {

struct alignas(8) RecJ {
    unsigned long long lo, hi;  // canonical (k-1)-mer
    unsigned int tag;           // oriented node id | side << 31 (side 0 = A: suffix, 1 = B: prefix)
    unsigned int pad;
};
static_assert(sizeof(RecJ) == 24, "join record layout");
__device__ inline unsigned int rec_bucket(const RecJ &r, int bbits) {
    return (unsigned int)(mix128(K128{r.lo, r.hi}) >> 32) >> (32 - bbits);
}
struct StoreJ {
    RecJ *p;
    __device__ inline RecJ load(uint64_t i) const { return p[i]; }
    __device__ inline void store(uint64_t i, const RecJ &r) const { p[i] = r; }
};
// minimizer-bucketed ids (count_wide.h, round 4): a junction's bucket = its own minimizer
// (pad = min_remix_w of it), which is the minimizer of most k-mers holding it -- a join bucket's
// nodes then sit in a few id ranges, so the link writes succ[x] stay local instead of spraying
// the whole node array (config 5: 3.9e8 random 4-B writes)
struct alignas(8) RecJM : RecJ {};
__device__ inline unsigned int rec_bucket(const RecJM &r, int bbits) { return bbits ? r.pad >> (32 - bbits) : 0u; }
struct StoreJM {
    RecJM *p;
    __device__ inline RecJM load(uint64_t i) const { return p[i]; }
    __device__ inline void store(uint64_t i, const RecJM &r) const { p[i] = r; }
};

// reverse complement of a j-mer, 32 <= j <= 62
__device__ inline K128 twin_j(const K128 &x, int j) {
    if (j <= 32) return K128{twin64(x.lo, j), 0ull};
    return twin128(x, j);
}

__device__ inline RecJ make_recj(const K128 &o, unsigned int node, unsigned int side) {
    RecJ r;
    r.lo = o.lo;
    r.hi = o.hi;
    r.tag = node | (side << 31);
    r.pad = 0;
    return r;
}

__global__ void __launch_bounds__(256) k_cursor_init(unsigned long long *gcur, uint64_t nb, uint64_t fcap) {
    for (uint64_t d = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; d < nb; d += (uint64_t)gridDim.x * blockDim.x)
        gcur[d] = d * fcap;
}

// per final bucket: group the records by (k-1)-mer in LDS, then write the links.  Slots are
// 24 B (key halves, one id word per side whose bit 31 marks a second distinct id): 2048 slots in
// 48 KB, three workgroups per CU.  ODD_K: no palindromic k-mers, twin(x) = x ^ 1 without the
// palindrome flags' random reads.
template <int SLOTS, int NT, bool ODD_K, typename R = RecJ>
__global__ void __launch_bounds__(NT) k_half_join(const R *recs, const unsigned long long *bbeg,
                                                  const unsigned long long *bend, const uint8_t *upal,
                                                  unsigned int *succ, unsigned int *overflow) {
    constexpr unsigned int MANY = 0x80000000u;
    __shared__ unsigned long long w1[SLOTS], w2[SLOTS];
    __shared__ unsigned int ids[2][SLOTS];
    __shared__ unsigned int s_over[2];
    const unsigned int b = blockIdx.x;
    for (int i = threadIdx.x; i < SLOTS; i += NT) {
        w1[i] = 0;
        w2[i] = 0;
        ids[0][i] = NONE32;
        ids[1][i] = NONE32;
    }
    if (threadIdx.x == 0) {
        s_over[0] = 0;
        s_over[1] = 0;
    }
    __syncthreads();
    const uint64_t r0 = bbeg[b], r1 = bend[b];
    for (uint64_t base = r0; base < r1; base += NT) {
        const uint64_t i = base + threadIdx.x;
        const bool valid = i < r1;
        R r{};
        if (valid) r = recs[i];
        const K128 o{r.lo, r.hi};
        const unsigned long long a1 = wide_w1(o), a2 = wide_w2(o);
        unsigned int slot = (unsigned int)(((uint64_t)(uint32_t)mix128(o) * SLOTS) >> 32);
        unsigned long long a = 0, bw = 0;
        bool miss = valid;
        if (valid) {
            a = w1[slot];
            bw = w2[slot];
            miss = !(a == a1 && bw == a2);
        }
        // claim by two CASes on the key's 63-bit halves (as lds_insert_w), wave-uniform loop
#pragma unroll 1
        while (__any(miss)) {
            if (miss) {
                if (a == 0) {
                    if (atomicAdd(&s_over[1], 1u) >= SLOTS - 1) {
                        s_over[0] = 1;
                        a = a1;
                        bw = a2;
                    } else {
                        a = atomicCAS(&w1[slot], 0ull, a1);
                        if (a == 0) a = a1;
                        else atomicSub(&s_over[1], 1u);
                    }
                }
                if (a == a1 && bw != a2) {
                    bw = w2[slot];
                    if (bw == 0) {
                        bw = atomicCAS(&w2[slot], 0ull, a2);
                        if (bw == 0) bw = a2;
                    }
                }
                if (!(a == a1 && bw == a2)) {
                    slot = slot + 1 == SLOTS ? 0u : slot + 1;
                    a = w1[slot];
                    bw = w2[slot];
                }
                miss = !(a == a1 && bw == a2);
            }
        }
        if (valid) {
            const unsigned int side = r.tag >> 31, id = r.tag & 0x7FFFFFFFu;
            const unsigned int old = atomicCAS(&ids[side][slot], NONE32, id);
            if (old != NONE32 && (old & ~MANY) != id) atomicOr(&ids[side][slot], MANY);
        }
    }
    __syncthreads();
    if (s_over[0]) {
        if (threadIdx.x == 0) atomicAdd(overflow, 1u);
        return;
    }
    for (int i = threadIdx.x; i < SLOTS; i += NT) {
        const unsigned int x = ids[0][i], y = ids[1][i];  // (NONE32 has bit 31 set too)
        if ((x | y) & MANY) continue;
        const unsigned int tx = ODD_K ? x ^ 1u : twin_node(upal, x), ty = ODD_K ? y ^ 1u : twin_node(upal, y);
        if (y == tx) continue;
        succ[x] = y;
        succ[ty] = tx;
    }
}

// ---- 64-bit keys (k <= 32): the same join on 16-B records --------------------------------------
// For the window-record count paths (k-mer-hash sub-tables: no minimizer locality for the
// neighbour probes) on large sets -- error-rich reads (1.3e7 solid keys), big genomes.
struct alignas(8) RecJ64 {
    unsigned long long key;  // canonical (k-1)-mer
    unsigned int tag;        // oriented node id | side << 31
    unsigned int pad;
};
static_assert(sizeof(RecJ64) == 16, "join record layout");
__device__ inline unsigned int rec_bucket(const RecJ64 &r, int bbits) {
    return (unsigned int)(mix64(r.key) >> 32) >> (32 - bbits);
}
struct StoreJ64 {
    RecJ64 *p;
    __device__ inline RecJ64 load(uint64_t i) const { return p[i]; }
    __device__ inline void store(uint64_t i, const RecJ64 &r) const { p[i] = r; }
};
__device__ inline RecJ64 make_recj64(unsigned long long o, unsigned int node, unsigned int side) {
    RecJ64 r;
    r.key = o;
    r.tag = node | (side << 31);
    r.pad = 0;
    return r;
}

// 16-B slots (key, one id word per side): 2048 slots in 32 KB
template <int SLOTS, int NT, bool ODD_K>
__global__ void __launch_bounds__(NT) k_half_join64(const RecJ64 *recs, const unsigned long long *bbeg,
                                                    const unsigned long long *bend, const uint8_t *upal,
                                                    unsigned int *succ, unsigned int *overflow) {
    constexpr unsigned int MANY = 0x80000000u;
    __shared__ unsigned long long kt[SLOTS];
    __shared__ unsigned int ids[2][SLOTS];
    __shared__ unsigned int s_over[2];
    const unsigned int b = blockIdx.x;
    for (int i = threadIdx.x; i < SLOTS; i += NT) {
        kt[i] = EMPTY_KEY;  // (a (k-1)-mer of <= 62 bits never equals it)
        ids[0][i] = NONE32;
        ids[1][i] = NONE32;
    }
    if (threadIdx.x == 0) {
        s_over[0] = 0;
        s_over[1] = 0;
    }
    __syncthreads();
    const uint64_t r0 = bbeg[b], r1 = bend[b];
    for (uint64_t base = r0; base < r1; base += NT) {
        const uint64_t i = base + threadIdx.x;
        const bool valid = i < r1;
        RecJ64 r{};
        if (valid) r = recs[i];
        unsigned int slot = (unsigned int)(((uint64_t)(uint32_t)mix64(r.key) * SLOTS) >> 32);
        unsigned long long cur = valid ? kt[slot] : 0ull;
        bool miss = valid && cur != r.key;
#pragma unroll 1
        while (__any(miss)) {
            if (miss) {
                if (cur == EMPTY_KEY) {
                    if (atomicAdd(&s_over[1], 1u) >= SLOTS - 1) {
                        s_over[0] = 1;
                        cur = r.key;
                    } else {
                        cur = atomicCAS(&kt[slot], EMPTY_KEY, r.key);
                        if (cur == EMPTY_KEY) cur = r.key;
                        else atomicSub(&s_over[1], 1u);
                    }
                }
                if (cur != r.key) {
                    slot = slot + 1 == SLOTS ? 0u : slot + 1;
                    cur = kt[slot];
                }
                miss = cur != r.key;
            }
        }
        if (valid) {
            const unsigned int side = r.tag >> 31, id = r.tag & 0x7FFFFFFFu;
            const unsigned int old = atomicCAS(&ids[side][slot], NONE32, id);
            if (old != NONE32 && (old & ~MANY) != id) atomicOr(&ids[side][slot], MANY);
        }
    }
    __syncthreads();
    if (s_over[0]) {
        if (threadIdx.x == 0) atomicAdd(overflow, 1u);
        return;
    }
    for (int i = threadIdx.x; i < SLOTS; i += NT) {
        const unsigned int x = ids[0][i], y = ids[1][i];
        if ((x | y) & MANY) continue;
        const unsigned int tx = ODD_K ? x ^ 1u : twin_node(upal, x), ty = ODD_K ? y ^ 1u : twin_node(upal, y);
        if (y == tx) continue;
        succ[x] = y;
        succ[ty] = tx;
    }
}

// ---- emit fused with the first level ----------------------------------------------------------
// The junction records go straight into the 2^lb1 first-level regions: each workgroup sorts
// its tile's records by region in LDS and stores them as runs reserved with one global atomic per
// region and tile (k_refine's scheme), so the level-1 pass over all 2U records disappears.  The
// rare second records of palindromic junctions take one global atomic each.
__device__ inline void half_recs(const K128 &c, unsigned int t, int j, const K128 &mj, const uint8_t *upal, RecJ &r1,
                                 RecJ &r2, bool &e1, bool &e2, RecJ &x1, RecJ &x2) {
    const unsigned int ic = 2u * t, itc = upal[t] ? ic : ic + 1u;
    const K128 s{c.lo & mj.lo, c.hi & mj.hi};
    const K128 p{(c.lo >> 2) | (c.hi << 62), c.hi >> 2};
    const K128 ts = twin_j(s, j), tp = twin_j(p, j);
    r1 = s < ts ? make_recj(s, ic, 0) : make_recj(ts, itc, 1);
    r2 = p < tp ? make_recj(p, ic, 1) : make_recj(tp, itc, 0);
    e1 = s == ts;
    e2 = p == tp;
    x1 = make_recj(s, ic, 0);
    x2 = make_recj(p, ic, 1);
}
__device__ inline void half_recs(unsigned long long c, unsigned int t, int j, unsigned long long mj,
                                 const uint8_t *upal, RecJ64 &r1, RecJ64 &r2, bool &e1, bool &e2, RecJ64 &x1,
                                 RecJ64 &x2) {
    const unsigned int ic = 2u * t, itc = upal[t] ? ic : ic + 1u;
    const unsigned long long s = c & mj, p = c >> 2;
    const unsigned long long ts = twin64(s, j), tp = twin64(p, j);
    r1 = s < ts ? make_recj64(s, ic, 0) : make_recj64(ts, itc, 1);
    r2 = p < tp ? make_recj64(p, ic, 1) : make_recj64(tp, itc, 0);
    e1 = s == ts;
    e2 = p == tp;
    x1 = make_recj64(s, ic, 0);
    x2 = make_recj64(p, ic, 1);
}
// the same records with their junctions' minimizers (k = j + 1 <= 63: the prefix junction holds
// m-mers 0 .. w - 2 of the key, the suffix junction m-mers 1 .. w - 1)
__device__ inline void half_recs(const K128 &c, unsigned int t, int j, const K128 &mj, const uint8_t *upal, RecJM &r1,
                                 RecJM &r2, bool &e1, bool &e2, RecJM &x1, RecJM &x2) {
    half_recs(c, t, j, mj, upal, static_cast<RecJ &>(r1), static_cast<RecJ &>(r2), e1, e2, static_cast<RecJ &>(x1),
              static_cast<RecJ &>(x2));
    const int k = j + 1, w = k - SK_M + 1;
    const K128 tc = twin128(c, k);
    uint32_t mp = 0xFFFFFFFFu, ms = 0xFFFFFFFFu;
    for (int p = 0; p < w; p++) {
        const uint32_t f = bits30_128(c, 2 * (k - SK_M - p)), r = bits30_128(tc, 2 * p);
        const uint32_t h = mmer_hash(f < r ? f : r);
        if (p < w - 1) mp = h < mp ? h : mp;
        if (p > 0) ms = h < ms ? h : ms;
    }
    const uint32_t vs = min_remix_w(ms), vp = min_remix_w(mp);
    r1.pad = vs;  // (r1 / x1: the suffix junction, r2 / x2: the prefix)
    x1.pad = vs;
    r2.pad = vp;
    x2.pad = vp;
}
__device__ inline K128 kmask_j(int j, K128 *) { return kmask128(j); }
__device__ inline unsigned long long kmask_j(int j, unsigned long long *) { return kmask64(j); }

template <typename K, typename R>
__global__ void __launch_bounds__(1024) k_half_emit_l1(const K *dkey, unsigned int U, int k, const uint8_t *upal,
                                                       int lb1, uint64_t fcap, unsigned long long *gcur, R *out,
                                                       unsigned int *over) {
    constexpr int NT = 1024, TILE = 2 * NT;
    __shared__ R tile[TILE];
    __shared__ uint8_t tj[TILE];
    __shared__ unsigned long long base[256];
    __shared__ unsigned int tcnt[256], tbeg[256], wsum[4];
    const int j = k - 1;
    const K mj = kmask_j(j, (K *)nullptr);
    const unsigned int F = 1u << lb1;
    for (uint64_t t0 = (uint64_t)blockIdx.x * NT; t0 < U; t0 += (uint64_t)gridDim.x * NT) {
        const uint64_t t = t0 + threadIdx.x;
        const bool valid = t < U;
        const unsigned int n = (unsigned int)min((uint64_t)NT, U - t0) * 2;
        if (threadIdx.x < 256) tcnt[threadIdx.x] = 0;
        __syncthreads();
        R r1{}, r2{}, x1{}, x2{};
        bool e1 = false, e2 = false;
        unsigned int j1 = 0, j2 = 0, k1 = 0, k2 = 0;
        if (valid) {
            half_recs(dkey[t], (unsigned int)t, j, mj, upal, r1, r2, e1, e2, x1, x2);
            j1 = rec_bucket(r1, lb1);
            j2 = rec_bucket(r2, lb1);
            k1 = atomicAdd(&tcnt[j1], 1u);
            k2 = atomicAdd(&tcnt[j2], 1u);
            if (e1) {  // (palindromic junctions: rare) one global atomic each
                const unsigned int jx = rec_bucket(x1, lb1);
                const unsigned long long pos = atomicAdd(&gcur[jx], 1ull);
                if (pos < (jx + 1ull) * fcap) out[pos] = x1;
                else *over = 1u;
            }
            if (e2) {
                const unsigned int jx = rec_bucket(x2, lb1);
                const unsigned long long pos = atomicAdd(&gcur[jx], 1ull);
                if (pos < (jx + 1ull) * fcap) out[pos] = x2;
                else *over = 1u;
            }
        }
        __syncthreads();
        unsigned long long mybase = 0;
        if (threadIdx.x < 256) {  // exclusive scan of the tile counts + run reservations
            const unsigned int v = threadIdx.x < F ? tcnt[threadIdx.x] : 0u;
            unsigned int incl = v;
            for (int o = 1; o < 64; o <<= 1) {
                const unsigned int u = __shfl_up(incl, o);
                if ((int)(threadIdx.x & 63) >= o) incl += u;
            }
            tbeg[threadIdx.x] = incl - v;
            if ((threadIdx.x & 63) == 63) wsum[threadIdx.x >> 6] = incl;
            if (v) mybase = atomicAdd(&gcur[threadIdx.x], (unsigned long long)v);
        }
        __syncthreads();
        if (threadIdx.x >= 64 && threadIdx.x < 256) {
            unsigned int add = 0;
            for (unsigned int w = 0; w < (threadIdx.x >> 6); w++) add += wsum[w];
            tbeg[threadIdx.x] += add;
        }
        __syncthreads();
        if (valid) {
            const unsigned int p1 = tbeg[j1] + k1, p2 = tbeg[j2] + k2;
            tile[p1] = r1;
            tj[p1] = (uint8_t)j1;
            tile[p2] = r2;
            tj[p2] = (uint8_t)j2;
        }
        if (threadIdx.x < 256) base[threadIdx.x] = mybase;
        __syncthreads();
        bool lost = false;
        for (unsigned int i = threadIdx.x; i < n; i += NT) {
            const unsigned int b = tj[i];
            const uint64_t pos = base[b] + (i - tbeg[b]);
            if (pos < (b + 1ull) * fcap) out[pos] = tile[i];
            else lost = true;
        }
        if (lost) *over = 1u;
        __syncthreads();
    }
}

}  // namespace ec
