// wide.h -- 128-bit k-mer keys for 32 < k <= 63 (BASELINE config 5: k = 51).
//
// K128 holds a 2k-bit code in (hi, lo), first base most significant, exactly the 64-bit
// algebra of common.h widened.  Counting uses one open-addressing HBM table whose slots
// claim a key with two 64-bit CASes: the key is split into two 63-bit halves, each stored
// with bit 63 set, so 0 marks an unclaimed word.  A thread claims / matches the first word,
// then the second; if another key with the same first half won the second word it moves on
// to the next slot.  Every slot whose first word is set gets its second word set by the
// same insert, so after the kernel the table is a plain key -> value map.  (k <= 63 keeps
// both halves to 63 bits.)
#pragma once
#include "window.h"

namespace ec {

struct K128 {
    unsigned long long lo, hi;
};

__host__ __device__ inline bool operator==(const K128 &a, const K128 &b) { return a.lo == b.lo && a.hi == b.hi; }
__host__ __device__ inline bool operator!=(const K128 &a, const K128 &b) { return !(a == b); }
__host__ __device__ inline bool operator<(const K128 &a, const K128 &b) {
    return a.hi < b.hi || (a.hi == b.hi && a.lo < b.lo);
}
__host__ __device__ inline bool operator<=(const K128 &a, const K128 &b) { return !(b < a); }

__host__ __device__ inline K128 kmask128(int k) {
    K128 m;
    m.lo = ~0ull;
    m.hi = k >= 64 ? ~0ull : ((1ull << (2 * k - 64)) - 1);
    return m;
}

// (x << 2 | b) & mask
__host__ __device__ inline K128 push128(K128 x, uint32_t b, const K128 &m) {
    K128 r;
    r.hi = ((x.hi << 2) | (x.lo >> 62)) & m.hi;
    r.lo = (x.lo << 2) | b;
    return r;
}

// reverse complement of a 2k-bit code (twin, referenceAssembler.py:7-10)
__host__ __device__ inline K128 twin128(K128 x, int k) {
    const K128 m = kmask128(k);
    const unsigned long long clo = x.lo ^ m.lo, chi = x.hi ^ m.hi;
    // reversed 128-bit value = (rev(lo) : rev(hi)), then shift right by 128 - 2k (> 0, < 64)
    const unsigned long long rh = rev2_64(clo), rl = rev2_64(chi);
    const int s = 128 - 2 * k;
    K128 r;
    r.lo = (rl >> s) | (rh << (64 - s));
    r.hi = rh >> s;
    return r;
}

__host__ __device__ inline uint64_t mix128(const K128 &x) { return mix64(x.lo ^ mix64(x.hi ^ 0x9E3779B97F4A7C15ull)); }

// base i (0 = first / most significant) of a k-mer
__host__ __device__ inline uint32_t base_at128(const K128 &x, int k, int i) {
    const int bit = 2 * (k - 1 - i);
    return (uint32_t)((bit >= 64 ? (x.hi >> (bit - 64)) : (x.lo >> bit)) & 3ull);
}

// the two claim words of a key (bit 63 set: never 0)
__device__ inline unsigned long long wide_w1(const K128 &c) { return (c.lo & 0x7FFFFFFFFFFFFFFFull) | (1ull << 63); }
__device__ inline unsigned long long wide_w2(const K128 &c) { return (c.lo >> 63) | (c.hi << 1) | (1ull << 63); }
__device__ inline K128 wide_key(unsigned long long w1, unsigned long long w2) {
    K128 c;
    c.lo = (w1 & 0x7FFFFFFFFFFFFFFFull) | ((w2 & 1ull) << 63);
    c.hi = (w2 & 0x7FFFFFFFFFFFFFFFull) >> 1;
    return c;
}

// 48-B slot: the two claim words, count, dense id, first events of canonical / twin string
struct alignas(16) SlotW {
    unsigned long long w1, w2;
    unsigned int count;
    unsigned int idx;
    unsigned long long fC, fT;
    unsigned long long pad;
};
static_assert(sizeof(SlotW) == 48, "wide slot layout");

// lookup sub-table slot of the partitioned wide count (count_wide.h k_bucket_w); id NONE =
// present, not solid
struct alignas(16) SubSlotW {
    unsigned long long w1, w2;
    unsigned int id, pad;
    unsigned long long pad2;
};
static_assert(sizeof(SubSlotW) == 32, "wide sub-table slot layout");

// exchange record of the multi-GPU path for k > 32 (ec_kmer_record_wide, 48 B)
struct alignas(16) AggW {
    unsigned long long lo, hi;
    unsigned int count, pad;
    unsigned long long fC, fT;
    unsigned long long pad2;
};
static_assert(sizeof(AggW) == 48, "wide record layout");

__global__ void __launch_bounds__(256) k_table_clear_w(SlotW *t, uint64_t cap) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < cap; i += (uint64_t)gridDim.x * blockDim.x) {
        SlotW s;
        s.w1 = 0;
        s.w2 = 0;
        s.count = 0;
        s.idx = NONE32;
        s.fC = NONE64;
        s.fT = NONE64;
        s.pad = 0;
        t[i] = s;
    }
}

// claim or find the slot of c; nullptr on probe overflow
__device__ inline SlotW *wide_slot(SlotW *table, uint64_t capmask, const K128 &c) {
    const unsigned long long w1 = wide_w1(c), w2 = wide_w2(c);
    uint64_t h = mix128(c) & capmask;
    for (int probe = 0; probe < MAX_PROBE; probe++) {
        SlotW *sl = table + h;
        unsigned long long a = sl->w1;
        if (a == 0) {
            a = atomicCAS(&sl->w1, 0ull, w1);
            if (a == 0) a = w1;
        }
        if (a == w1) {
            unsigned long long b = sl->w2;
            if (b == 0) {
                b = atomicCAS(&sl->w2, 0ull, w2);
                if (b == 0) b = w2;
            }
            if (b == w2) return sl;
        }
        h = (h + 1) & capmask;
    }
    return nullptr;
}

__device__ inline unsigned int lookup_w(const SlotW *table, uint64_t capmask, const K128 &c) {
    const unsigned long long w1 = wide_w1(c), w2 = wide_w2(c);
    uint64_t h = mix128(c) & capmask;
    for (int probe = 0; probe < MAX_PROBE; probe++) {
        const unsigned long long a = table[h].w1;
        if (a == 0) return NONE32;
        if (a == w1 && table[h].w2 == w2) return table[h].idx;
        h = (h + 1) & capmask;
    }
    return NONE32;
}

// windows of read r in reference insertion order, 128-bit codes (for_each_window widened)
template <typename Fn>
__device__ inline void for_each_window_w(ByteReader &rd, uint64_t s, uint64_t len, int k, uint64_t r, Fn &&fn) {
    const K128 mask = kmask128(k);
    const int sh = 2 * (k - 1);  // >= 64
    uint32_t wb = 0;
    uint64_t p = 0;
    while (p < len) {
        uint64_t q = p;
        while (q < len && base_code(rd(s + q)) < 4) q++;
        if (q - p >= (uint64_t)k) {
            const uint32_t m = (uint32_t)(q - p - k + 1);
            K128 fwd{0, 0}, rc{0, 0};
            for (uint64_t t = p; t < q; t++) {
                const uint32_t b = base_code(rd(s + t));
                fwd = push128(fwd, b, mask);
                rc.lo = (rc.lo >> 2) | (rc.hi << 62);
                rc.hi = (rc.hi >> 2) | ((unsigned long long)(3u - b) << (sh - 64));
                if (t - p + 1 >= (uint64_t)k) {
                    const uint32_t i = (uint32_t)(t - p + 1 - k);
                    fn(fwd, rc, (r << 32) | (uint64_t)(2 * wb + i), (r << 32) | (uint64_t)(2 * wb + 2 * m - 1 - i));
                }
            }
            wb += m;
        }
        p = q + 1;
    }
}

// prescan: positions, first invalid byte, HyperLogLog registers (2^HLL_BITS, merged with
// atomicMax) of the canonical keys -- sizes the table
__global__ void __launch_bounds__(256) k_prescan_w(const uint8_t *buf, const uint64_t *off, uint64_t nreads, int k,
                                                   unsigned int *hll, unsigned long long *npos,
                                                   unsigned long long *bad) {
    __shared__ unsigned int reg[HLL_M];
    for (int i = threadIdx.x; i < HLL_M; i += blockDim.x) reg[i] = 0;
    __syncthreads();
    unsigned long long np = 0;
    for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < nreads; r += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t s = off[r], len = off[r + 1] - s;
        ByteReader rd(buf);
        for (uint64_t t = 0; t < len; t++)
            if (base_code(rd(s + t)) == 5) {
                atomicMin(bad, (unsigned long long)(s + t));
                break;
            }
        for_each_window_w(rd, s, len, k, 0, [&](const K128 &f, const K128 &rc, uint64_t, uint64_t) {
            const K128 c = f < rc ? f : rc;
            const uint64_t h = mix128(c);
            const unsigned int j = (unsigned int)(h >> (64 - HLL_BITS));
            const unsigned int rho = (unsigned int)__clzll((long long)((h << HLL_BITS) | (1ull << (HLL_BITS - 1)))) + 1;
            atomicMax(&reg[j], rho);
            np++;
        });
    }
    for (int o = 32; o > 0; o >>= 1) np += __shfl_xor(np, o);
    if ((threadIdx.x & 63) == 0 && np) atomicAdd(npos, np);
    __syncthreads();
    for (int i = threadIdx.x; i < HLL_M; i += blockDim.x)
        if (reg[i]) atomicMax(&hll[i], reg[i]);
}

// count (thread per read), semantics of k_count (count_global.h)
__global__ void __launch_bounds__(256) k_count_w(const uint8_t *buf, const uint64_t *off, uint64_t nreads, int k,
                                                 SlotW *table, uint64_t capmask, unsigned int *overflow,
                                                 uint64_t read_base) {
    for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < nreads; r += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t s = off[r], len = off[r + 1] - s;
        ByteReader rd(buf);
        for_each_window_w(rd, s, len, k, r + read_base, [&](const K128 &f, const K128 &rc, uint64_t ef, uint64_t er) {
            const bool pal = f == rc;
            const K128 c = f < rc ? f : rc;
            uint64_t eC = f <= rc ? ef : er;
            uint64_t eT = f <= rc ? er : ef;
            if (pal) eC = eT = ef;
            SlotW *sl = wide_slot(table, capmask, c);
            if (!sl) {
                atomicOr(overflow, 1u);
                return;
            }
            atomicAdd(&sl->count, pal ? 2u : 1u);
            if (eC < sl->fC) atomicMin(&sl->fC, (unsigned long long)eC);
            if (eT < sl->fT) atomicMin(&sl->fT, (unsigned long long)eT);
        });
    }
}

// merge exchanged records (sum of counts, min of first events)
__global__ void __launch_bounds__(256) k_merge_agg_w(const AggW *in, uint64_t n, SlotW *table, uint64_t capmask,
                                                     unsigned int *overflow) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < n; t += (uint64_t)gridDim.x * blockDim.x) {
        const AggW a = in[t];
        if (a.lo == ~0ull && a.hi == ~0ull) continue;  // all-gather filler record
        const K128 c{a.lo, a.hi};
        SlotW *sl = wide_slot(table, capmask, c);
        if (!sl) {
            atomicOr(overflow, 1u);
            continue;
        }
        if (a.count) atomicAdd(&sl->count, a.count);
        if (a.fC < sl->fC) atomicMin(&sl->fC, a.fC);
        if (a.fT < sl->fT) atomicMin(&sl->fT, a.fT);
    }
}

// HyperLogLog registers (2^bits u32) of the records' keys: the merge table is sized by the
// distinct keys, not by the records -- an owner's received records repeat each key once per
// source (config 5: 2e8 records of 2.5e7 keys a rank; the streaming count's folds ~3x)
__global__ void __launch_bounds__(256) k_hll_aggw(const AggW *in, uint64_t n, int bits, unsigned int *reg) {
    __shared__ unsigned int s[1 << 12];
    const unsigned int M = 1u << bits;
    for (unsigned int i = threadIdx.x; i < M; i += blockDim.x) s[i] = 0;
    __syncthreads();
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < n; t += (uint64_t)gridDim.x * blockDim.x) {
        const AggW a = in[t];
        if (a.lo == ~0ull && a.hi == ~0ull) continue;  // all-gather filler record
        const uint64_t h = mix128(K128{a.lo, a.hi});
        const unsigned int j = (unsigned int)(h >> (64 - bits));
        const unsigned int rho = (unsigned int)__clzll((long long)((h << bits) | (1ull << (bits - 1)))) + 1u;
        if (rho > s[j]) atomicMax(&s[j], rho);
    }
    __syncthreads();
    for (unsigned int i = threadIdx.x; i < M; i += blockDim.x)
        if (s[i]) atomicMax(&reg[i], s[i]);
}

// dense arrays -> exchange records, grouped by owner rank (multi-GPU, k > 32)
__device__ inline unsigned int owner_of_w(const K128 &c, unsigned int nowners) {
    return (unsigned int)(((mix128(c) >> 32) * (uint64_t)nowners) >> 32);
}

}  // namespace ec
