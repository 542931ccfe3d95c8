// shard.h -- building blocks of the read-sharded multi-GPU path (distributed.py):
//   every rank counts its read shard (phase_count, no solid filter), exports its distinct
//   k-mers grouped by owner rank (owner = hash of the canonical key), the records are
//   exchanged with one RCCL all-to-all, each owner merges what it received (sum of counts,
//   min of first events) and applies the solid filter; the solid sets are all-gathered and
//   every rank runs the graph phase on the full set.
#pragma once
#include "count_global.h"
#include "wide.h"
#include "count_part.h"
#include "graph.h"

namespace ec {

// one aggregated canonical k-mer: the payload of the exchange (ec_kmer_record in eulerhip.h)
struct alignas(16) Agg {
    unsigned long long key;
    unsigned int count;
    unsigned int pad;
    unsigned long long fC;
    unsigned long long fT;
};
static_assert(sizeof(Agg) == 32, "agg layout");

__device__ inline unsigned int owner_of(uint64_t key, unsigned int nowners) {
    return (unsigned int)(((mix64(key ^ 0xD6E8FEB86659FD93ull) >> 32) * (uint64_t)nowners) >> 32);
}

constexpr int MAX_OWNERS = 256;

__device__ inline unsigned int owner_of(const K128 &c, unsigned int nowners) { return owner_of_w(c, nowners); }

// The owner rule of the exchange.  For SK_MIN_K <= k <= 32 a key's owner is the range of its
// minimizer (superkmer.h minimizer_of, uniform 32 bits after min_remix), and the merge and the
// gathered-set load bucket keys by the same minimizer (SolidIndex::sk): an owner's merged set
// -- and so its segment of the gathered dense ids -- comes out in bucket order, a node's
// neighbours mostly share its bucket, and the partitioned links / ranking touch the lookup
// sub-tables and node arrays with the locality of the one-GPU path.  128-bit keys with
// 33 <= k <= 52 (round 5): the range of the key's 128-bit minimizer (graph.h minimizer_of_w, the
// count_wide.h bucket minimizer), and the owner merge emits its set in minimizer order
// (order_by_minimizer_w), so config 5's gathered ids have the same locality and take the
// partitioned finish.  Other k: a key hash.
struct OwnerFn {
    MinCfg mc;
    int sk;
    int wk = 0;  // 128-bit keys: k when owners are minimizer ranges, 0 for key-hash owners
    __device__ inline unsigned int operator()(unsigned long long key, unsigned int n) const {
        return sk ? (unsigned int)(((uint64_t)minimizer_of(key, mc) * n) >> 32) : owner_of(key, n);
    }
    __device__ inline unsigned int operator()(const K128 &key, unsigned int n) const {
        return wk ? (unsigned int)(((uint64_t)minimizer_of_w(key, wk) * n) >> 32) : owner_of(key, n);
    }
};

// owner merge of 128-bit keys on minimizer owners: the dense set reordered by placement
// (minimizer << 32 | low half of mix128, graph.h wide_place), each minimizer's first id marked
// in bmark for the partitioned finish's tile plan (k_tile_plan)
__global__ void __launch_bounds__(256) k_wplace(const K128 *dkey, unsigned int U, int k, unsigned long long *place,
                                                unsigned int *idx) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < U; t += (uint64_t)gridDim.x * blockDim.x) {
        place[t] = wide_place(dkey[t], k, true);
        idx[t] = (unsigned int)t;
    }
}
__global__ void __launch_bounds__(256) k_wpermute(const unsigned int *perm, unsigned int U, const K128 *ik,
                                                  const unsigned int *ic, const unsigned long long *ifc,
                                                  const unsigned long long *ift, K128 *ok, unsigned int *oc,
                                                  unsigned long long *ofc, unsigned long long *oft) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < U; t += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned int j = perm[t];
        ok[t] = ik[j];
        oc[t] = ic[j];
        ofc[t] = ifc[j];
        oft[t] = ift[j];
    }
}
// one thread per 32 ids: bit i of bmark set iff id i starts a minimizer (sorted placements)
__global__ void __launch_bounds__(256) k_wmarks(const unsigned long long *place, unsigned int U, unsigned int *bmark,
                                                unsigned int words) {
    for (uint64_t w = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; w < words; w += (uint64_t)gridDim.x * blockDim.x) {
        unsigned int m = 0;
        for (unsigned int b = 0; b < 32; b++) {
            const uint64_t i = w * 32 + b;
            if (i < U && (i == 0 || (place[i] >> 32) != (place[i - 1] >> 32))) m |= 1u << b;
        }
        bmark[w] = m;
    }
}

// the exchange record of a key type: Agg (64-bit keys) or AggW (K128)
template <typename K> struct RecOf;
template <> struct RecOf<unsigned long long> {
    using T = Agg;
    __device__ static inline Agg make(unsigned long long k, unsigned int c, unsigned long long fc, unsigned long long ft) {
        Agg a;
        a.key = k;
        a.count = c;
        a.pad = 0;
        a.fC = fc;
        a.fT = ft;
        return a;
    }
};
template <> struct RecOf<K128> {
    using T = AggW;
    __device__ static inline AggW make(const K128 &k, unsigned int c, unsigned long long fc, unsigned long long ft) {
        AggW a;
        a.lo = k.lo;
        a.hi = k.hi;
        a.count = c;
        a.pad = 0;
        a.fC = fc;
        a.fT = ft;
        a.pad2 = 0;
        return a;
    }
};

// Owner-major export in two passes without global atomics (a cursor per owner hit by every
// block serialised at the memory side: 223 us for 4.6 M records at one owner).
// Chunk b = records [b OWN_CHUNK, (b + 1) OWN_CHUNK): bh[o * nblk + b] = its records of owner o;
// after an inclusive scan of bh (owner-major) chunk b's owner-o records start at
// bh_incl[o * nblk + b - 1] -- the owner's offset in the export included.
constexpr unsigned int OWN_CHUNK = 8192;

template <typename K>
__global__ void __launch_bounds__(256) k_owner_hist(const K *dkey, unsigned int n, unsigned int nowners,
                                                    unsigned int nblk, unsigned int *bh, OwnerFn own,
                                                    unsigned int *oid, const unsigned long long *dfc = nullptr,
                                                    const unsigned long long *dft = nullptr,
                                                    unsigned int *evmax = nullptr) {
    __shared__ unsigned int h[MAX_OWNERS];
    __shared__ unsigned int s_mx[2];
    for (unsigned int i = threadIdx.x; i < nowners; i += blockDim.x) h[i] = 0;
    if (threadIdx.x < 2) s_mx[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t c0 = (uint64_t)blockIdx.x * OWN_CHUNK, c1 = min<uint64_t>(c0 + OWN_CHUNK, n);
    unsigned int mr = 0, ml = 0;  // largest shard-relative read id / window position of the events
    for (uint64_t t = c0 + threadIdx.x; t < c1; t += blockDim.x) {
        const unsigned int o = own(dkey[t], nowners);  // kept for the scatter (a minimizer is ~250 VALU)
        oid[t] = o;
        atomicAdd(&h[o], 1u);
        if (evmax) {
            const unsigned long long a = dfc[t], b = dft[t];
            if (a != NONE64) mr = max(mr, (unsigned int)(a >> 32)), ml = max(ml, (unsigned int)a);
            if (b != NONE64) mr = max(mr, (unsigned int)(b >> 32)), ml = max(ml, (unsigned int)b);
        }
    }
    if (evmax) {
        for (int o = 32; o > 0; o >>= 1) mr = max(mr, (unsigned int)__shfl_xor(mr, o)), ml = max(ml, (unsigned int)__shfl_xor(ml, o));
        if ((threadIdx.x & 63) == 0) atomicMax(&s_mx[0], mr), atomicMax(&s_mx[1], ml);
    }
    __syncthreads();
    for (unsigned int i = threadIdx.x; i < nowners; i += blockDim.x) bh[(uint64_t)i * nblk + blockIdx.x] = h[i];
    if (evmax && threadIdx.x == 0) atomicMax(&evmax[0], s_mx[0]), atomicMax(&evmax[1], s_mx[1]);
}

// ---- compact exchange records (round 5) ---------------------------------------------------------
// The all-to-all carries every rank's distinct k-mers (config 4: 4.6 M per rank whatever N is).
// Events of a shard count are shard-relative, (read << 32) | window position, with reads <
// 2^24 and positions < 2^9 at the bench's shapes, so a record carries them as 32-bit
// (read << lf_bits) | lf (0xFFFFFFFF: no event) and the receiver adds the source's global read
// base: 20-B records (k <= 32; 28 B for 128-bit keys) instead of 32 / 48 B.  A rank whose events
// do not fit sends full records (lf_bits -1); the receiver decodes per source.
struct CRec {
    uint32_t w[5];  // key lo, key hi, count, eC, eT
};
struct CRecW {
    uint32_t w[7];  // key lo.lo, lo.hi, hi.lo, hi.hi, count, eC, eT
};
static_assert(sizeof(CRec) == 20 && sizeof(CRecW) == 28, "compact record layout");
template <typename K> struct CRecOf;
template <> struct CRecOf<unsigned long long> {
    using T = CRec;
    static constexpr int KW = 2;
};
template <> struct CRecOf<K128> {
    using T = CRecW;
    static constexpr int KW = 4;
};
__device__ inline void key_words(unsigned long long k, uint32_t *w) { w[0] = (uint32_t)k, w[1] = (uint32_t)(k >> 32); }
__device__ inline void key_words(const K128 &k, uint32_t *w) {
    w[0] = (uint32_t)k.lo, w[1] = (uint32_t)(k.lo >> 32), w[2] = (uint32_t)k.hi, w[3] = (uint32_t)(k.hi >> 32);
}
__device__ inline uint32_t ev_pack(unsigned long long e, int lfb) {
    return e == NONE64 ? 0xFFFFFFFFu : (uint32_t)(((e >> 32) << lfb) | (e & 0xFFFFFFFFull));
}
__device__ inline unsigned long long ev_unpack(uint32_t v, int lfb, unsigned long long read_base) {
    if (v == 0xFFFFFFFFu) return NONE64;
    return ((read_base + (v >> lfb)) << 32) | (v & ((1u << lfb) - 1u));
}

template <typename K>
__global__ void __launch_bounds__(256) k_owner_scatter_c(const K *dkey, const unsigned int *dcnt,
                                                         const unsigned long long *dfc, const unsigned long long *dft,
                                                         unsigned int n, unsigned int nowners, unsigned int nblk,
                                                         const unsigned int *bh_incl, typename CRecOf<K>::T *out,
                                                         int lfb, const unsigned int *oid) {
    constexpr int KW = CRecOf<K>::KW;
    __shared__ unsigned int h[MAX_OWNERS];
    __shared__ unsigned int base[MAX_OWNERS];
    for (unsigned int i = threadIdx.x; i < nowners; i += blockDim.x) {
        const uint64_t j = (uint64_t)i * nblk + blockIdx.x;
        h[i] = 0;
        base[i] = j ? bh_incl[j - 1] : 0u;
    }
    __syncthreads();
    const uint64_t c0 = (uint64_t)blockIdx.x * OWN_CHUNK, c1 = min<uint64_t>(c0 + OWN_CHUNK, n);
    for (uint64_t t = c0 + threadIdx.x; t < c1; t += blockDim.x) {
        const unsigned int o = oid[t];
        const unsigned int rk = atomicAdd(&h[o], 1u);
        typename CRecOf<K>::T r;
        key_words(dkey[t], r.w);
        r.w[KW] = dcnt[t];
        r.w[KW + 1] = ev_pack(dfc[t], lfb);
        r.w[KW + 2] = ev_pack(dft[t], lfb);
        out[base[o] + rk] = r;
    }
}

// received records of every source -> exchange records with global events (the merge's input);
// source s: records [roff[s], roff[s + 1]) at byte boffs[s], compact (lfb[s] >= 0) or full
template <typename K>
__global__ void __launch_bounds__(256) k_uncompact(const uint8_t *in, const unsigned long long *boff,
                                                   const unsigned long long *roff, const long long *rbase,
                                                   const int *lfb, int nsrc, uint64_t n,
                                                   typename RecOf<K>::T *out) {
    using R = typename RecOf<K>::T;
    using C = typename CRecOf<K>::T;
    constexpr int KW = CRecOf<K>::KW;
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < n; t += (uint64_t)gridDim.x * blockDim.x) {
        int a = 0, b = nsrc;  // roff[a] <= t < roff[b]
        while (b - a > 1) {
            const int m = (a + b) >> 1;
            if (t >= roff[m]) a = m;
            else b = m;
        }
        const uint64_t i = t - roff[a];
        if (lfb[a] < 0) {  // full records (word copies: a source segment is 4-B aligned only)
            const uint32_t *src = reinterpret_cast<const uint32_t *>(in + boff[a]) + i * (sizeof(R) / 4);
            uint32_t *dst = reinterpret_cast<uint32_t *>(out + t);
#pragma unroll
            for (int q = 0; q < (int)(sizeof(R) / 4); q++) dst[q] = src[q];
            continue;
        }
        const C c = reinterpret_cast<const C *>(in + boff[a])[i];
        K key;
        if constexpr (KW == 2) key = (unsigned long long)c.w[0] | (unsigned long long)c.w[1] << 32;
        else key = K128{(unsigned long long)c.w[0] | (unsigned long long)c.w[1] << 32,
                        (unsigned long long)c.w[2] | (unsigned long long)c.w[3] << 32};
        out[t] = RecOf<K>::make(key, c.w[KW], ev_unpack(c.w[KW + 1], lfb[a], (unsigned long long)rbase[a]),
                                ev_unpack(c.w[KW + 2], lfb[a], (unsigned long long)rbase[a]));
    }
}

// The received records read in place (round 5, k <= 32): record t's source by a search over
// roff, compact records decoded with their source's read base.  The owner merge's bucket ids and
// bucket tables read them directly (XAggSource) instead of a decoded copy (k_uncompact wrote and
// read back 147 MB a rank at 8 weak ranks: 55 us + the gather of 32-B records).
struct XIn {
    const uint8_t *in;
    const unsigned long long *boff, *roff;
    const long long *rbase;
    const int *lfb;
    int nsrc;
    __device__ inline int src_of(uint64_t t) const {
        int a = 0, b = nsrc;  // roff[a] <= t < roff[b]
        while (b - a > 1) {
            const int m = (a + b) >> 1;
            if (t >= roff[m]) a = m;
            else b = m;
        }
        return a;
    }
    __device__ inline Agg get(uint64_t t) const {
        const int a = src_of(t);
        const uint64_t i = t - roff[a];
        const int lb = lfb[a];
        const uint32_t *w = reinterpret_cast<const uint32_t *>(in + boff[a]);  // (4-B aligned only)
        Agg r;
        if (lb < 0) {
            uint32_t *d = reinterpret_cast<uint32_t *>(&r);
#pragma unroll
            for (int q = 0; q < (int)(sizeof(Agg) / 4); q++) d[q] = w[i * (sizeof(Agg) / 4) + q];
            return r;
        }
        const uint32_t *c = w + i * 5;
        const unsigned long long rb = (unsigned long long)rbase[a];
        r = RecOf<unsigned long long>::make((unsigned long long)c[0] | (unsigned long long)c[1] << 32, c[2],
                                            ev_unpack(c[3], lb, rb), ev_unpack(c[4], lb, rb));
        return r;
    }
    __device__ inline unsigned long long key(uint64_t t) const {
        const int a = src_of(t);
        const uint64_t i = t - roff[a];
        const uint32_t *w = reinterpret_cast<const uint32_t *>(in + boff[a]) + i * (lfb[a] < 0 ? sizeof(Agg) / 4 : 5);
        return (unsigned long long)w[0] | (unsigned long long)w[1] << 32;
    }
};
static_assert(sizeof(CRec) == 20, "XIn decodes 5-word records");
struct PlainIn {
    const Agg *p;
    __device__ inline unsigned long long key(uint64_t t) const { return p[t].key; }
};

// scatter dense records into owner-major order at the scanned chunk bases (owners from
// k_owner_hist's oid); evbase = the
// shard's first global read id << 32 (ec_count_shard counts shard-relative)
template <typename K>
__global__ void __launch_bounds__(256) k_owner_scatter(const K *dkey, const unsigned int *dcnt,
                                                       const unsigned long long *dfc, const unsigned long long *dft,
                                                       unsigned int n, unsigned int nowners, unsigned int nblk,
                                                       const unsigned int *bh_incl, typename RecOf<K>::T *out,
                                                       unsigned long long evbase, const unsigned int *oid) {
    __shared__ unsigned int h[MAX_OWNERS];
    __shared__ unsigned int base[MAX_OWNERS];
    for (unsigned int i = threadIdx.x; i < nowners; i += blockDim.x) {
        const uint64_t j = (uint64_t)i * nblk + blockIdx.x;
        h[i] = 0;
        base[i] = j ? bh_incl[j - 1] : 0u;
    }
    __syncthreads();
    const uint64_t c0 = (uint64_t)blockIdx.x * OWN_CHUNK, c1 = min<uint64_t>(c0 + OWN_CHUNK, n);
    for (uint64_t t = c0 + threadIdx.x; t < c1; t += blockDim.x) {
        const K key = dkey[t];
        const unsigned int o = oid[t];
        const unsigned int rk = atomicAdd(&h[o], 1u);
        // shard-relative first events -> global (NONE64 = no event, kept)
        const unsigned long long fc = dfc[t], ft = dft[t];
        out[base[o] + rk] = RecOf<K>::make(key, dcnt[t], fc == NONE64 ? fc : fc + evbase, ft == NONE64 ? ft : ft + evbase);
    }
}

// owner side: aggregate received records into the HBM table (count sum, first-event min)
__global__ void __launch_bounds__(256) k_merge_agg(const Agg *in, uint64_t n, Slot *table, uint64_t capmask,
                                                   unsigned int *overflow) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < n; t += (uint64_t)gridDim.x * blockDim.x) {
        const Agg a = in[t];
        if (a.key == EMPTY_KEY) continue;  // all-gather filler record (never a canonical key)
        uint64_t h = mix64(a.key) & capmask;
        for (int probe = 0;; probe++) {
            if (probe >= MAX_PROBE) {
                atomicOr(overflow, 1u);
                break;
            }
            Slot *sl = table + h;
            unsigned long long cur = sl->key;
            if (cur == EMPTY_KEY) {
                cur = atomicCAS(&sl->key, EMPTY_KEY, a.key);
                if (cur == EMPTY_KEY) cur = a.key;
            }
            if (cur == a.key) {
                atomicAdd(&sl->count, a.count);
                if (a.fC < sl->fC) atomicMin(&sl->fC, a.fC);
                if (a.fT < sl->fT) atomicMin(&sl->fT, a.fT);
                break;
            }
            h = (h + 1) & capmask;
        }
    }
}

// evbase: after ec_count_shard the first events are shard-relative (+ read_base << 32 makes them
// global, as k_owner_scatter does); after a merge they are global already (evbase 0)
template <typename K>
__global__ void __launch_bounds__(256) k_export_dense(const K *dkey, const unsigned int *dcnt,
                                                      const unsigned long long *dfc, const unsigned long long *dft,
                                                      unsigned int n, typename RecOf<K>::T *out,
                                                      unsigned long long evbase) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < n; t += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned long long fc = dfc[t], ft = dft[t];
        out[t] = RecOf<K>::make(dkey[t], dcnt[t], fc == NONE64 ? fc : fc + evbase, ft == NONE64 ? ft : ft + evbase);
    }
}


// ---- bucketed merge: exchange records -> LDS bucket tables (k_bucket over AggSource) -------
// bucket id = top bbits of mix64(key) (the fused path's bucket hash, so the SolidIndex
// sub-table layout is shared), or with sk the top bbits of the key's minimizer (OwnerFn);
// filler records (all-ones key) go to bucket 2^bbits, past the end.
template <typename In>
__global__ void __launch_bounds__(256) k_agg_bucket_ids(In in, uint64_t n, int bbits, unsigned int *bid, MinCfg mc,
                                                        int sk) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < n; t += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned long long key = in.key(t);
        bid[t] = key == EMPTY_KEY ? (1u << bbits)
                 : sk             ? sk_bucket_of(minimizer_of(key, mc), bbits)
                                  : (bbits ? (unsigned int)(mix64(key) >> (64 - bbits)) : 0u);
    }
}

// Counting sort of record indices by bucket id (round 4; a rocPRIM radix sort of (id, index)
// pairs took 4 x 55 us a call).  Round 5: per chunk of CS_CHUNK records an LDS histogram whose
// nonzero bins are added to job-wide bin totals (k_cs_hist), one exclusive scan of the nbins
// totals (k_cs_starts: the bin starts and the scatter cursors), and per chunk the histogram
// again, each nonzero bin's range reserved with one global atomic and the indices placed
// through LDS cursors (k_cs_scatter).  Round 4 stored the per-chunk histograms bin-major and
// scanned all nbins x chunks cells: 8193 bins x 281 chunks, written and read back at a stride
// of one cell per chunk, cost the owner merge 46 + 21 + 64 us.  The order inside a bin is not
// deterministic -- the bucket tables do not depend on it.  1024 threads a chunk (256 left ~280
// workgroups on 256 CUs for 4.6 M records).
constexpr unsigned int CS_CHUNK = 16384;
__global__ void __launch_bounds__(1024) k_cs_hist(const unsigned int *bid, uint64_t n, unsigned int nbins,
                                                 unsigned int *tot) {
    extern __shared__ unsigned int csh[];
    for (unsigned int i = threadIdx.x; i < nbins; i += blockDim.x) csh[i] = 0;
    __syncthreads();
    const uint64_t t0 = (uint64_t)blockIdx.x * CS_CHUNK, t1 = t0 + CS_CHUNK < n ? t0 + CS_CHUNK : n;
    for (uint64_t t = t0 + threadIdx.x; t < t1; t += blockDim.x) atomicAdd(&csh[bid[t]], 1u);
    __syncthreads();
    for (unsigned int i = threadIdx.x; i < nbins; i += blockDim.x)
        if (csh[i]) atomicAdd(&tot[i], csh[i]);
}
// excl = exclusive scan of tot (scan_incl_u32 gives incl): bin starts (u64) and cursors
// (end: bstart[nbins] = n as well)
__global__ void __launch_bounds__(256) k_cs_starts(const unsigned int *tot, const unsigned int *incl, unsigned int nbins,
                                                   unsigned long long *bstart, unsigned int *cur, bool end) {
    if (end && blockIdx.x == 0 && threadIdx.x == 0) bstart[nbins] = incl[nbins - 1];
    for (unsigned int b = blockIdx.x * blockDim.x + threadIdx.x; b < nbins; b += gridDim.x * blockDim.x) {
        const unsigned int e = incl[b] - tot[b];
        bstart[b] = e;
        cur[b] = e;
    }
}
__global__ void __launch_bounds__(1024) k_cs_scatter(const unsigned int *bid, uint64_t n, unsigned int nbins,
                                                    unsigned int *cur, unsigned int *out) {
    extern __shared__ unsigned int csh[];
    for (unsigned int i = threadIdx.x; i < nbins; i += blockDim.x) csh[i] = 0;
    __syncthreads();
    const uint64_t t0 = (uint64_t)blockIdx.x * CS_CHUNK, t1 = t0 + CS_CHUNK < n ? t0 + CS_CHUNK : n;
    for (uint64_t t = t0 + threadIdx.x; t < t1; t += blockDim.x) atomicAdd(&csh[bid[t]], 1u);
    __syncthreads();
    for (unsigned int i = threadIdx.x; i < nbins; i += blockDim.x) {
        const unsigned int c = csh[i];
        if (c) csh[i] = atomicAdd(&cur[i], c);  // this chunk's range of bin i
    }
    __syncthreads();
    for (uint64_t t = t0 + threadIdx.x; t < t1; t += blockDim.x) out[atomicAdd(&csh[bid[t]], 1u)] = (unsigned int)t;
}

// bstart[b] = first position of bucket b in the sorted ids (b = 0..nb; bstart[nb] = real records)
__global__ void __launch_bounds__(256) k_bucket_bounds(const unsigned int *sbid, uint64_t n, unsigned int nb,
                                                       unsigned long long *bstart) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const long long b = sbid[i], pb = i ? (long long)sbid[i - 1] : -1;
        for (long long q = pb + 1; q <= b && q <= (long long)nb; q++) bstart[q] = i;
        if (i + 1 == n)
            for (long long q = b + 1; q <= (long long)nb; q++) bstart[q] = n;
    }
}

// first probe slot in the bucket table: mix64 (sks = 0) or, for minimizer buckets, the top sks
// bits of sk_slot (SolidIndex::slot0 with sk = 1, slots = 2^sks)
#define EC_AGG_SOURCE                                                                               \
    __device__ inline void seg(uint32_t, uint32_t) {}                                                \
    __device__ inline unsigned long long key_out(unsigned long long c) const { return c; }           \
    __device__ inline uint64_t slot_hash(unsigned long long c) const {                               \
        return sks ? (uint64_t)(sk_slot(c) >> (32 - sks)) : mix64(c);                                \
    }

struct AggSource {
    EC_AGG_SOURCE
    const Agg *in;
    const unsigned int *perm;
    int sks;
    using Raw = Agg;
    static constexpr bool kDet = false;
    __device__ inline Raw fetch(uint64_t i) const { return in[perm[i]]; }
    __device__ inline unsigned int id(const Raw &) const { return 0; }
    __device__ inline void decode(const Agg &a, unsigned long long &key, unsigned int &add, unsigned long long &eC,
                                  unsigned long long &eT) const {
        key = a.key;
        add = a.count;
        eC = a.fC;
        eT = a.fT;
    }
};


// AggSource over the received records in place (XIn)
struct XAggSource {
    EC_AGG_SOURCE
    XIn in;
    const unsigned int *perm;
    int sks;
    using Raw = Agg;
    static constexpr bool kDet = false;
    __device__ inline Raw fetch(uint64_t i) const { return in.get(perm[i]); }
    __device__ inline unsigned int id(const Raw &) const { return 0; }
    __device__ inline void decode(const Agg &a, unsigned long long &key, unsigned int &add, unsigned long long &eC,
                                  unsigned long long &eT) const {
        key = a.key;
        add = a.count;
        eC = a.fC;
        eT = a.fT;
    }
};

// ---- partitioned graph phase (k <= 32): every rank loads the all-gathered solid set with the
// SAME dense ids (position among the non-filler records, i.e. owner-major), computes the links
// of its own owner segment only, and the successor arrays are all-gathered.
struct AggDet {
    Agg a;
    unsigned int id;
};
struct AggDetSource {
    EC_AGG_SOURCE
    const Agg *in;
    const unsigned int *perm;
    const unsigned int *ids;  // dense id of each record (NONE for fillers, which sort past the end)
    int sks;
    using Raw = AggDet;
    static constexpr bool kDet = true;
    __device__ inline Raw fetch(uint64_t i) const {
        const unsigned int j = perm[i];
        AggDet r;
        r.a = in[j];
        r.id = ids[j];
        return r;
    }
    __device__ inline unsigned int id(const Raw &r) const { return r.id; }
    __device__ inline void decode(const AggDet &r, unsigned long long &key, unsigned int &add, unsigned long long &eC,
                                  unsigned long long &eT) const {
        key = r.a.key;
        add = r.a.count;
        eC = r.a.fC;
        eT = r.a.fT;
    }
};

constexpr unsigned int DET_CHUNK = 8192;
// non-filler records (all-gather filler: all-ones bytes)
__device__ inline bool det_valid(const Agg &r) { return r.key != EMPTY_KEY; }
__device__ inline bool det_valid(const AggW &r) { return !(r.lo == ~0ull && r.hi == ~0ull); }

template <typename R>
__global__ void __launch_bounds__(256) k_det_count(const R *in, uint64_t n, unsigned int *bc) {
    const uint64_t c0 = (uint64_t)blockIdx.x * DET_CHUNK;
    const uint64_t c1 = c0 + DET_CHUNK < n ? c0 + DET_CHUNK : n;
    unsigned int v = 0;
    for (uint64_t i = c0 + threadIdx.x; i < c1; i += blockDim.x) v += det_valid(in[i]);
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    __shared__ unsigned int ws[4];
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) bc[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}
// bs = inclusive scan of the chunk counts; ids[i] = rank of record i among the non-fillers
template <typename R>
__global__ void __launch_bounds__(256) k_det_ids(const R *in, uint64_t n, const unsigned int *bs, unsigned int *ids) {
    __shared__ unsigned int wsum[4];
    const uint64_t c0 = (uint64_t)blockIdx.x * DET_CHUNK;
    const uint64_t c1 = c0 + DET_CHUNK < n ? c0 + DET_CHUNK : n;
    unsigned int base = blockIdx.x ? bs[blockIdx.x - 1] : 0u;
    const unsigned int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (uint64_t i0 = c0; i0 < c1; i0 += blockDim.x) {
        const uint64_t i = i0 + threadIdx.x;
        const bool valid = i < c1 && det_valid(in[i]);
        const unsigned long long m = __ballot(valid);
        if (lane == 0) wsum[wid] = (unsigned int)__popcll(m);
        __syncthreads();
        unsigned int off = base;
        for (unsigned int q = 0; q < wid; q++) off += wsum[q];
        if (i < c1) ids[i] = valid ? off + (unsigned int)__popcll(m & ((1ull << lane) - 1)) : NONE32;
        base += wsum[0] + wsum[1] + wsum[2] + wsum[3];
        __syncthreads();
    }
}

// partitioned graph phase for k > 32: record i of the gathered set -> dense id ids[i] (dense
// arrays in gathered order) + the key's slot in the HBM lookup table (gathered keys are
// distinct: one writer per slot)
__global__ void __launch_bounds__(256) k_load_det_w(const AggW *in, uint64_t n, const unsigned int *ids, SlotW *table,
                                                   uint64_t capmask, K128 *dkey, unsigned int *dcnt,
                                                   unsigned long long *dfc, unsigned long long *dft,
                                                   unsigned int *overflow) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < n; t += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned int id = ids[t];
        if (id == NONE32) continue;
        const AggW a = in[t];
        const K128 c{a.lo, a.hi};
        dkey[id] = c;
        dcnt[id] = a.count;
        dfc[id] = a.fC;
        dft[id] = a.fT;
        SlotW *sl = wide_slot(table, capmask, c);
        if (!sl) {
            atomicOr(overflow, 1u);
            continue;
        }
        sl->idx = id;
    }
}

}  // namespace ec
