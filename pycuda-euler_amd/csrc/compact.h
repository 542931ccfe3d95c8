// compact.h -- deterministic table -> dense-array compaction for the HBM tables (Slot, SlotW):
// per-chunk counts, one scan, then a write pass that ranks solid slots within the chunk by
// wave ballots.  Dense ids follow table order; no contended global counter (a per-wave
// atomic on one word serialises at the memory side, ~88 per us).
#pragma once
#include "count_global.h"
#include "wide.h"

namespace ec {

constexpr unsigned int COMPACT_CHUNK = 16384;

__device__ inline bool slot_present(const Slot &s) { return s.key != EMPTY_KEY; }
__device__ inline bool slot_present(const SlotW &s) { return s.w1 != 0; }
__device__ inline void slot_key(const Slot &s, unsigned long long *dkey, unsigned int u) { dkey[u] = s.key; }
__device__ inline void slot_key(const SlotW &s, K128 *dkey, unsigned int u) { dkey[u] = wide_key(s.w1, s.w2); }

template <typename SlotT>
__global__ void __launch_bounds__(256) k_compact_count(const SlotT *table, uint64_t cap, long long limit,
                                                       unsigned int *bc, unsigned long long *ndistinct) {
    const uint64_t c0 = (uint64_t)blockIdx.x * COMPACT_CHUNK;
    const uint64_t c1 = c0 + COMPACT_CHUNK < cap ? c0 + COMPACT_CHUNK : cap;
    unsigned int ns = 0, np = 0;
    for (uint64_t i = c0 + threadIdx.x; i < c1; i += blockDim.x) {
        const SlotT s = table[i];
        const bool p = slot_present(s);
        np += p;
        ns += p && (long long)s.count > limit;
    }
    for (int o = 32; o > 0; o >>= 1) {
        ns += __shfl_xor(ns, o);
        np += __shfl_xor(np, o);
    }
    __shared__ unsigned int ws[4], wp[4];
    if ((threadIdx.x & 63) == 0) {
        ws[threadIdx.x >> 6] = ns;
        wp[threadIdx.x >> 6] = np;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        bc[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
        const unsigned int p = wp[0] + wp[1] + wp[2] + wp[3];
        if (p) atomicAdd(ndistinct, (unsigned long long)p);
    }
}

// bs = inclusive scan of the chunk counts
template <typename SlotT, typename KeyT>
__global__ void __launch_bounds__(256) k_compact_write(SlotT *table, uint64_t cap, long long limit,
                                                       const unsigned int *bs, KeyT *dkey, unsigned int *dcnt,
                                                       unsigned long long *dfc, unsigned long long *dft) {
    __shared__ unsigned int wsum[4];
    const uint64_t c0 = (uint64_t)blockIdx.x * COMPACT_CHUNK;
    const uint64_t c1 = c0 + COMPACT_CHUNK < cap ? c0 + COMPACT_CHUNK : cap;
    unsigned int base = blockIdx.x ? bs[blockIdx.x - 1] : 0u;
    const unsigned int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (uint64_t i0 = c0; i0 < c1; i0 += blockDim.x) {
        const uint64_t i = i0 + threadIdx.x;
        SlotT s;
        bool solid = false;
        if (i < c1) {
            s = table[i];
            solid = slot_present(s) && (long long)s.count > limit;
        }
        const unsigned long long m = __ballot(solid);
        if (lane == 0) wsum[wid] = (unsigned int)__popcll(m);
        __syncthreads();
        unsigned int off = base;
        for (unsigned int q = 0; q < wid; q++) off += wsum[q];
        const unsigned int tot = wsum[0] + wsum[1] + wsum[2] + wsum[3];
        if (solid) {
            const unsigned int u = off + (unsigned int)__popcll(m & ((1ull << lane) - 1));
            slot_key(s, dkey, u);
            dcnt[u] = s.count;
            dfc[u] = s.fC;
            dft[u] = s.fT;
            table[i].idx = u;
        }
        base += tot;
        __syncthreads();
    }
}

__global__ void k_compact_total(const unsigned int *bs, unsigned int nblk, unsigned int *nsolid) {
    *nsolid = bs[nblk - 1];
}

}  // namespace ec
