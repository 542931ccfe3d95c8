// count_global.h -- general counting path: one open-addressing table in HBM, 64-bit CAS
// insert, atomic count and first-event minima per window.  Used when the partitioned LDS
// path does not apply (distinct k-mers per bucket beyond the LDS table, reads > 32 kbp).
#pragma once
#include "window.h"

namespace ec {
// ---------------------------------------------------------------------------------------
// hash slot: 32 B, one per distinct canonical k-mer.  key + count + dense id + the first
// insertion event of the canonical string (fC) and of its twin (fT).
struct alignas(32) Slot {
    unsigned long long key;
    unsigned int count;
    unsigned int idx;
    unsigned long long fC;
    unsigned long long fT;
};
static_assert(sizeof(Slot) == 32, "slot layout");

// HyperLogLog estimate (harmonic mean + small-range correction) from the merged registers
__global__ void __launch_bounds__(1024) k_hll_final(const unsigned int *reg, int mbits, double *est) {
    const int M = 1 << mbits;
    __shared__ double red[1024];
    __shared__ int zeros[1024];
    double sum = 0;
    int z = 0;
    for (int j = threadIdx.x; j < M; j += blockDim.x) {
        const uint32_t m = reg[j];
        sum += ldexp(1.0, -(int)m);
        z += (m == 0);
    }
    red[threadIdx.x] = sum;
    zeros[threadIdx.x] = z;
    __syncthreads();
    for (int o = blockDim.x / 2; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) {
            red[threadIdx.x] += red[threadIdx.x + o];
            zeros[threadIdx.x] += zeros[threadIdx.x + o];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const double m = M;
        const double alpha = 0.7213 / (1.0 + 1.079 / m);
        double e = alpha * m * m / red[0];
        if (e <= 2.5 * m && zeros[0] > 0) e = m * log(m / (double)zeros[0]);
        *est = e;
    }
}

// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_table_clear(Slot *t, uint64_t cap) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < cap; i += (uint64_t)gridDim.x * blockDim.x) {
        Slot s;
        s.key = EMPTY_KEY;
        s.count = 0;
        s.idx = NONE32;
        s.fC = NONE64;
        s.fT = NONE64;
        t[i] = s;
    }
}

// count: thread per read.  Reference semantics: d[km] += 1 for every forward window and for
// every window of twin(seg) (build:31-35) == +1 per window on the canonical key, +2 when the
// window is its own twin (even-k palindrome: both loops hit the same string).
__global__ void __launch_bounds__(256) k_count(const uint8_t *buf, const uint64_t *off, uint64_t nreads, int k,
                                               Slot *table, uint64_t capmask, unsigned int *overflow,
                                               uint64_t read_base) {
    for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < nreads;
         r += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t s = off[r], len = off[r + 1] - s;
        ByteReader rd(buf);
        for_each_window(rd, s, len, k, r + read_base, [&](uint64_t fwd, uint64_t rc, uint64_t ef, uint64_t er) {
            const bool pal = fwd == rc;
            const uint64_t c = fwd < rc ? fwd : rc;
            // first events of the canonical string and of its twin
            uint64_t eC = fwd <= rc ? ef : er;
            uint64_t eT = fwd <= rc ? er : ef;
            if (pal) eC = eT = ef;
            uint64_t h = mix64(c) & capmask;
            for (int probe = 0;; probe++) {
                if (probe >= MAX_PROBE) {
                    atomicOr(overflow, 1u);
                    return;
                }
                Slot *sl = table + h;
                unsigned long long cur = sl->key;
                if (cur == EMPTY_KEY) {
                    cur = atomicCAS(&sl->key, EMPTY_KEY, (unsigned long long)c);
                    if (cur == EMPTY_KEY) cur = c;
                }
                if (cur == c) {
                    atomicAdd(&sl->count, pal ? 2u : 1u);
                    if (eC < sl->fC) atomicMin(&sl->fC, (unsigned long long)eC);
                    if (eT < sl->fT) atomicMin(&sl->fT, (unsigned long long)eT);
                    return;
                }
                h = (h + 1) & capmask;
            }
        });
    }
}

__device__ inline unsigned int lookup(const Slot *table, uint64_t capmask, uint64_t c) {
    uint64_t h = mix64(c) & capmask;
    for (int probe = 0; probe < MAX_PROBE; probe++) {
        const unsigned long long kk = table[h].key;
        if (kk == c) return table[h].idx;
        if (kk == EMPTY_KEY) return NONE32;
        h = (h + 1) & capmask;
    }
    return NONE32;
}

}  // namespace ec
