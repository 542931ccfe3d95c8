// count_part.h -- partitioned k-mer counting (the production path of build:25-42).
//
// Instead of one HBM hash table hit by a global atomic per k-mer position, the positions
// are radix-partitioned by the top bits of mix64(canonical key) into B buckets and each
// bucket is counted in a 2048-slot hash table in LDS by one workgroup:
//
//   k_upsweep    per read group : LDS-staged reads -> windows -> alphabet check, P,
//                                 HyperLogLog registers, 4096-way fine histogram
//   (host)                      : B = 2^bbits from the distinct estimate (<= ~1024 keys per bucket)
//   k_coarse     per (bucket,group): coarse counts, bucket-major; exclusive scan -> offsets
//   k_downsweep  per read group : windows again -> 16-B records {key, read, local events}
//                                 scattered to their (bucket, group) run
//   k_bucket     per bucket     : records -> LDS table (CAS insert, count += 1|2, 64-bit
//                                 atomicMin of first events) -> solid filter (count > limit,
//                                 build:37-39) -> dense arrays + the bucket's lookup sub-table
//
// Record = {u64 canonical key, u32 read, u32 lC | lT << 16}: the first events of the canonical
// string and of its twin are (read << 32) | lC and (read << 32) | lT (window.h); a window is its
// own twin (even-k palindrome, counted twice by build) iff lC == lT.  Local events < 2^16 limit
// this path to reads of < 32768 windows; longer reads take the general path (count_global.h).
#pragma once
#include "window.h"

namespace ec {

constexpr int FINE_BITS = 13;
constexpr int FINE = 1 << FINE_BITS;       // fine histogram bins = max buckets
constexpr int HLL_REG_BITS = 11;           // HyperLogLog registers (top 11 hash bits, 2.3% error)
constexpr int TILE_READS = 256;            // reads staged per tile (one per thread)
constexpr int STAGE_BYTES = 28672;         // LDS staging per tile
constexpr int BUCKET_THREADS = 1024;
constexpr int MAX_COARSE_BITS = 9;         // downsweep writes <= 512 bucket runs per group
constexpr int REFINE_TILE = 4096;          // records per refine tile (64 KiB of LDS)
constexpr int REFINE_FANOUT = 256;         // final buckets per coarse bucket
constexpr unsigned int MAX_LOCAL_EVENT = 65535;

struct alignas(16) Rec {
    unsigned long long key;
    unsigned int read;
    unsigned int ev;  // lC | lT << 16
};
static_assert(sizeof(Rec) == 16, "record layout");

// Compact 12-B record for N-free reads of one length L (the common short-read case):
// meta = read << (ibits + 1) | o << ibits | i, with i the window index (< m = L - k + 1 <=
// 2^ibits) and o = 1 when the canonical string is the window's twin.  The local events are
// then lC = o ? 2m-1-i : i and lT = o ? i : 2m-1-i (a palindrome: both i), as in window.h.
struct Rec12 {
    unsigned int klo, khi, meta;
};
static_assert(sizeof(Rec12) == 12, "compact record layout");

__device__ inline unsigned long long rkey(const Rec &r) { return r.key; }
__device__ inline unsigned long long rkey(const Rec12 &r) { return ((unsigned long long)r.khi << 32) | r.klo; }
// final bucket of a window record: top bbits of mix64(key) (bbits >= 1)
// (the high word alone: the compiler then skips the low half of the 64-bit product)
__device__ inline unsigned int rec_bucket(const Rec &r, int bbits) {
    return (unsigned int)(mix64(r.key) >> 32) >> (32 - bbits);
}
__device__ inline unsigned int rec_bucket(const Rec12 &r, int bbits) {
    return (unsigned int)(mix64(rkey(r)) >> 32) >> (32 - bbits);
}

// record construction in the downsweep: window (fwd, rc) of read r with local events lf / lr
struct MakeRec {
    uint64_t read_base;
    __device__ inline Rec operator()(uint64_t fwd, uint64_t rc, uint32_t lf, uint32_t lr, uint64_t r) const {
        uint32_t lC = fwd <= rc ? lf : lr, lT = fwd <= rc ? lr : lf;
        if (fwd == rc) lT = lC = lf;
        Rec rec;
        rec.key = fwd < rc ? fwd : rc;
        rec.read = (unsigned int)(r + read_base);
        rec.ev = lC | (lT << 16);
        return rec;
    }
};
struct MakeRec12 {
    uint64_t read_base;
    int ibits;
    __device__ inline Rec12 operator()(uint64_t fwd, uint64_t rc, uint32_t lf, uint32_t, uint64_t r) const {
        const uint64_t c = fwd < rc ? fwd : rc;
        Rec12 rec;
        rec.klo = (unsigned int)c;
        rec.khi = (unsigned int)(c >> 32);
        rec.meta = ((unsigned int)(r + read_base) << (ibits + 1)) | ((fwd <= rc ? 0u : 1u) << ibits) | lf;
        return rec;
    }
};

// solid lookup sub-table slot (bucket region of `slots` slots); id NONE = present, not solid
struct alignas(16) SubSlot {
    unsigned long long key;
    unsigned int id;
    unsigned int pad;
};

// record stores: 16-B records in one array; compact records as split arrays (8-B keys,
// 4-B meta) so every access is an aligned, coalesced dwordx2 / dword.  Measured (10M x 100 bp):
// k_bucket runs 1.6x longer over compact records (same instruction and LDS counts, half the
// resident waves -- not understood), so the refine widens them back to 16 B (Store12to16):
// compact records then save 25 % of the downsweep write and the refine read.
struct Store16 {
    Rec *p;
    __device__ inline Rec load(uint64_t i) const { return p[i]; }
    __device__ inline void store(uint64_t i, const Rec &r) const { p[i] = r; }
};
// refine output of compact records widened back to 16-B records (lC | lT events), so that
// k_bucket reads the 16-B layout it runs fastest on
struct Store12to16 {
    Rec *p;
    int ibits;
    int k;
    unsigned int m2;  // 2m - 1
    __device__ inline void store(uint64_t i, const Rec12 &r) const {
        const unsigned long long key = rkey(r);
        const unsigned int w = r.meta & ((1u << ibits) - 1), o = (r.meta >> ibits) & 1u;
        unsigned int lC = o ? m2 - w : w, lT = o ? w : m2 - w;
        if (!(k & 1) && twin64(key, k) == key) lC = lT = w;  // even-k palindrome
        Rec out;
        out.key = key;
        out.read = r.meta >> (ibits + 1);
        out.ev = lC | (lT << 16);
        p[i] = out;
    }
};

// compact records as one packed 12-B array (the refine output read by k_bucket)
struct Store12P {
    unsigned int *p;
    __device__ inline void store(uint64_t i, const Rec12 &r) const {
        p[3 * i] = r.klo;
        p[3 * i + 1] = r.khi;
        p[3 * i + 2] = r.meta;
    }
};

struct Store12 {
    unsigned long long *key;
    unsigned int *meta;
    __device__ inline Rec12 load(uint64_t i) const {
        const unsigned long long k = key[i];
        Rec12 r;
        r.klo = (unsigned int)k;
        r.khi = (unsigned int)(k >> 32);
        r.meta = meta[i];
        return r;
    }
    __device__ inline void store(uint64_t i, const Rec12 &r) const {
        key[i] = rkey(r);
        meta[i] = r.meta;
    }
};

// LDS byte reader over a staged tile (slow path: reads with 'N')
struct LdsReader {
    const uint8_t *lds;
    uint64_t base;  // buffer offset of lds[0]
    __device__ inline uint32_t operator()(uint64_t pos) const { return lds[pos - base]; }
};

// Stage reads [r0, r1) of the tile into LDS (coalesced 16-B loads from the 16-B aligned
// absolute address below the first byte).  Returns false when the tile does not fit.
__device__ inline bool stage_tile(const uint8_t *buf, const uint64_t *off, uint64_t r0, uint64_t r1,
                                  uint8_t *stage, uint64_t &base) {
    const uint64_t b0 = off[r0], b1 = off[r1];
    const uint64_t a0 = ((uint64_t)(buf + b0)) & ~15ull;
    const uint64_t a1 = (((uint64_t)(buf + b1)) + 15) & ~15ull;
    if (a1 - a0 > (uint64_t)STAGE_BYTES) return false;
    base = a0 - (uint64_t)buf;
    const uint4 *src = reinterpret_cast<const uint4 *>(a0);
    uint4 *dst = reinterpret_cast<uint4 *>(stage);
    const unsigned n16 = (unsigned)((a1 - a0) >> 4);
    for (unsigned i = threadIdx.x; i < n16; i += blockDim.x) dst[i] = src[i];
    return true;
}

// For every read of the group (one read per thread, TILE_READS-read tiles staged in LDS):
// fn(staged, LdsRead, LdsReader, read, offset, len).  `staged` = false when a tile's bytes
// exceed the stage (long reads): the callback then reads global memory.
struct NoHook {
    __device__ inline void operator()(uint64_t) const {}
};

template <typename Fn, typename Pre = NoHook, typename Post = NoHook>
__device__ inline void for_group_reads(const uint8_t *buf, const uint64_t *off, uint64_t g0, uint64_t g1,
                                       uint8_t *stage, Fn &&fn, Pre pre = Pre(), Post post = Post()) {
    for (uint64_t r0 = g0; r0 < g1; r0 += TILE_READS) {
        const uint64_t r1 = min(r0 + TILE_READS, g1);
        uint64_t base = 0;
        __syncthreads();  // previous tile fully consumed
        pre(r0 / TILE_READS);
        const bool staged = stage_tile(buf, off, r0, r1, stage, base);
        __syncthreads();
        const uint64_t r = r0 + threadIdx.x;
        if (r < r1) {
            const uint64_t s = off[r], len = off[r + 1] - s;
            const uint64_t rel = s - base;
            LdsRead rv{reinterpret_cast<const uint32_t *>(stage), (uint32_t)(rel >> 2), (uint32_t)(rel & 3)};
            LdsReader lr{stage, base};
            fn(staged, rv, lr, r, s, len);
        }
        __syncthreads();
        post(r0 / TILE_READS);
    }
}

__device__ inline uint64_t group_begin(uint64_t g, uint64_t gsize, uint64_t nreads) {
    return min(g * gsize, nreads);
}

// ---- upsweep: alphabet + P + HLL + fine histogram per read group -------------------------
// fine bins are packed 2 x u16 per LDS word; a bin reaching 65535 sets *skew (the host then
// takes the general path: one k-mer repeated > 65535 times inside one read group)
__global__ void __launch_bounds__(TILE_READS) k_upsweep(const uint8_t *buf, const uint64_t *off, uint64_t nreads,
                                                       int k, uint64_t gsize, unsigned int *hist, uint8_t *hll_blocks,
                                                       unsigned long long *npos, unsigned long long *bad,
                                                       unsigned int *maxlocal, unsigned int *skew,
                                                       unsigned int *lens) {
    __shared__ __attribute__((aligned(16))) uint8_t stage[STAGE_BYTES + 16];
    __shared__ unsigned int h_cnt[FINE / 2];
    __shared__ unsigned int h_reg[1 << HLL_REG_BITS];
    for (int i = threadIdx.x; i < FINE / 2; i += blockDim.x) h_cnt[i] = 0;
    for (int i = threadIdx.x; i < (1 << HLL_REG_BITS); i += blockDim.x) h_reg[i] = 0;
    const uint64_t g = blockIdx.x;
    const uint64_t g0 = group_begin(g, gsize, nreads), g1 = group_begin(g + 1, gsize, nreads);
    unsigned long long mypos = 0;
    unsigned int mymax = 0, mylmax = 0, mylmin = 0xFFFFFFFFu, mynonclean = 0;
    // (rho from the 21 hash bits under the register index: registers saturate at 22, far
    // above log2(distinct / 2048) for any input that fits one GPU)
    auto win = [&](uint64_t fwd, uint64_t rc) {
        const uint64_t c = fwd < rc ? fwd : rc;
        const uint32_t hh = (uint32_t)(mix64(c) >> 32);
        const uint32_t j = hh >> (32 - HLL_REG_BITS);
        const uint32_t rho = (uint32_t)__clz((int)((hh << HLL_REG_BITS) | (1u << (HLL_REG_BITS - 1)))) + 1;
        const uint32_t f = hh >> (32 - FINE_BITS);
        atomicAdd(&h_cnt[f >> 1], 1u << ((f & 1) * 16));  // overflow: checked after the group
        if (rho > h_reg[j]) atomicMax(&h_reg[j], rho);
    };
    for_group_reads(buf, off, g0, g1, stage,
                    [&](bool staged, const LdsRead &rv, const LdsReader &lr, uint64_t r, uint64_t s, uint64_t len) {
        uint32_t flags = 3;
        if (staged) flags = read_flags(rv, (uint32_t)len);
        if (flags == 0) {  // N-free read: one segment
            if (len >= (uint64_t)k) {
                const uint32_t m = (uint32_t)(len - k + 1);
                mylmax = max(mylmax, (uint32_t)len);
                mylmin = min(mylmin, (uint32_t)len);
                windows_clean(rv, (uint32_t)len, k, [&](uint64_t fwd, uint64_t rc, uint32_t) { win(fwd, rc); });
                mypos += m;
                mymax = max(mymax, 2 * m - 1);
            }
            return;
        }
        mynonclean = 1;
        auto slow = [&](auto &rd) {
            for (uint64_t t = 0; t < len; t++) {
                if (base_code(rd(s + t)) == 5) {
                    atomicMin(bad, (unsigned long long)(s + t));
                    break;
                }
            }
            mypos += for_each_window(rd, s, len, k, r, [&](uint64_t fwd, uint64_t rc, uint64_t ef, uint64_t er) {
                win(fwd, rc);
                const uint32_t le = max((uint32_t)ef, (uint32_t)er);
                mymax = max(mymax, le);
            });
        };
        if (staged) {
            LdsReader l2 = lr;
            slow(l2);
        } else {
            ByteReader br(buf);
            slow(br);
        }
    });
    // a u16 bin that wrapped (one k-mer > 65535 times in the group) lowers the sum of the bins
    // below the group's window count (65535 per carry into the neighbour, 65536 per wrap out)
    unsigned long long binsum = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < FINE / 2; i += blockDim.x) binsum += (h_cnt[i] & 0xFFFFu) + (h_cnt[i] >> 16);
    for (int o = 32; o > 0; o >>= 1) {
        mypos += __shfl_down(mypos, o);
        binsum += __shfl_down(binsum, o);
        mymax = max(mymax, (unsigned int)__shfl_down(mymax, o));
        mylmax = max(mylmax, (unsigned int)__shfl_down(mylmax, o));
        mylmin = min(mylmin, (unsigned int)__shfl_down(mylmin, o));
        mynonclean |= (unsigned int)__shfl_down(mynonclean, o);
    }
    __shared__ unsigned long long s_diff;
    if (threadIdx.x == 0) s_diff = 0;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&s_diff, mypos - binsum);  // mod 2^64: 0 iff no bin overflowed
        if (mypos) atomicAdd(npos, mypos);
        if (mymax) atomicMax(maxlocal, mymax);
        if (mylmax) atomicMax(&lens[0], mylmax);
        if (mylmin != 0xFFFFFFFFu) atomicMax(&lens[1], ~mylmin);  // lens[1] = ~(min length)
        if (mynonclean) atomicOr(&lens[2], 1u);
    }
    __syncthreads();
    if (threadIdx.x == 0 && s_diff != 0) atomicOr(skew, 1u);
    for (int i = threadIdx.x; i < FINE; i += blockDim.x) hist[g * FINE + i] = (h_cnt[i >> 1] >> ((i & 1) * 16)) & 0xFFFFu;
    for (int i = threadIdx.x; i < (1 << HLL_REG_BITS); i += blockDim.x)
        hll_blocks[g * (1 << HLL_REG_BITS) + i] = (uint8_t)h_reg[i];
}

// coarse counts, bucket-major: cnt[c * ngroups + g] = group g's records in coarse bucket c
// (sum of its fine bins; a read group is one downsweep workgroup, which fills its runs in order)
// FB = fine histogram bits (FINE_BITS; count_wide.h uses FINE_W_BITS)
template <int FB = FINE_BITS>
__global__ void __launch_bounds__(256) k_coarse(const unsigned int *hist, uint64_t ngroups, int cbits,
                                                unsigned long long *cnt) {
    constexpr int FINE = 1 << FB;
    const uint64_t C = 1ull << cbits;
    const int per = 1 << (FB - cbits);
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < C * ngroups;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t c = i / ngroups, g = i % ngroups;
        const unsigned int *h = hist + g * FINE + c * per;
        unsigned long long sum = 0;
        for (int j = 0; j < per; j++) sum += h[j];
        cnt[i] = sum;
    }
}

// fine-bin totals over all groups (2-D: bins x group slices, one atomic per slice) and the
// HyperLogLog register maxima over all groups
constexpr int TOT_SLICES = 32;
template <int FB = FINE_BITS>
__global__ void __launch_bounds__(256) k_fine_totals(const unsigned int *hist, const uint8_t *hll, uint64_t ngroups,
                                                     unsigned long long *ftot, unsigned int *hreg,
                                                     unsigned long long *total = nullptr) {
    constexpr int FINE = 1 << FB;
    const unsigned int f = blockIdx.x * blockDim.x + threadIdx.x;  // < FINE
    const unsigned int sl = blockIdx.y;
    unsigned long long sum = 0;
    unsigned int mx = 0;
    for (uint64_t g = sl; g < ngroups; g += TOT_SLICES) {
        sum += hist[g * FINE + f];
        if (f < (1u << HLL_REG_BITS)) mx = max(mx, (unsigned int)hll[g * (1 << HLL_REG_BITS) + f]);
    }
    if (sum) atomicAdd(&ftot[f], sum);
    if (f < (1u << HLL_REG_BITS) && mx) atomicMax(&hreg[f], mx);
    if (total) {  // (the records of all bins: one atomic per wave)
        unsigned long long w = sum;
        for (int o = 32; o > 0; o >>= 1) w += __shfl_down(w, o);
        if ((threadIdx.x & 63) == 0 && w) atomicAdd(total, w);
    }
}

// records per final bucket (bbits granularity); tot[B] = 0 so its exclusive scan ends at P
template <int FB = FINE_BITS>
__global__ void __launch_bounds__(256) k_bucket_totals(const unsigned long long *ftot, int bbits,
                                                       unsigned long long *tot) {
    const uint64_t B = 1ull << bbits;
    const int per = 1 << (FB - bbits);
    for (uint64_t b = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; b <= B; b += (uint64_t)gridDim.x * blockDim.x) {
        unsigned long long sum = 0;
        if (b < B)
            for (int i = 0; i < per; i++) sum += ftot[b * per + i];
        tot[b] = sum;
    }
}

// ---- downsweep: records to their (coarse bucket, tile) run --------------------------------
// N-free reads (the bulk) are processed in lock-step batches of DS_R windows per thread; each
// batch (2048 records) is counting-sorted by coarse bucket in LDS and stored as contiguous
// runs, so a wave's stores cover a few full lines instead of 64 scattered 16-B pieces.
// Reads with 'N' (and tiles too long to stage) follow after the batches, storing directly.
constexpr int DS_R = 8;
constexpr int DS_BATCH = TILE_READS * DS_R;
constexpr int DS_MAX_CBITS = 8;

template <typename RecT, typename Make, typename Store>
__global__ void __launch_bounds__(TILE_READS) k_downsweep(const uint8_t *buf, const uint64_t *off, uint64_t nreads,
                                                         int k, uint64_t gsize, uint64_t ngroups, int cbits,
                                                         const unsigned long long *offs, Store recs, Make mk) {
    __shared__ __attribute__((aligned(16))) uint8_t stage[STAGE_BYTES + 16];
    __shared__ RecT sorted[DS_BATCH];
    __shared__ uint8_t sbk[DS_BATCH];
    __shared__ unsigned int bcnt[1 << DS_MAX_CBITS], bbeg[1 << DS_MAX_CBITS];
    __shared__ unsigned long long cur[1 << DS_MAX_CBITS], gbase[1 << DS_MAX_CBITS];
    __shared__ unsigned int s_rounds, s_total, s_wave[TILE_READS / 64];
    const uint64_t g = blockIdx.x;
    const int C = 1 << cbits;
    const unsigned int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const uint64_t mask = kmask64(k);
    const int sh = 2 * (k - 1);
    const uint64_t g0 = group_begin(g, gsize, nreads), g1 = group_begin(g + 1, gsize, nreads);
    auto make = [&](uint64_t fwd, uint64_t rc, uint32_t lf, uint32_t lr, uint64_t r, unsigned int &cb) {
        const uint64_t c = fwd < rc ? fwd : rc;
        cb = cbits ? ((unsigned int)(mix64(c) >> 32) >> (32 - cbits)) : 0u;  // high word only
        return mk(fwd, rc, lf, lr, r);
    };
    for (uint64_t r0 = g0; r0 < g1; r0 += TILE_READS) {
        const uint64_t r1 = min(r0 + TILE_READS, g1);
        __syncthreads();
        for (int c = tid; c < C; c += TILE_READS) {
            if (r0 == g0) cur[c] = offs[(uint64_t)c * ngroups + g];  // the group's run of coarse bucket c
            bcnt[c] = 0;
        }
        if (tid == 0) s_rounds = 0;
        uint64_t base = 0;
        const bool staged = stage_tile(buf, off, r0, r1, stage, base);
        __syncthreads();
        const uint64_t r = r0 + tid;
        const bool valid = r < r1;
        uint64_t s = 0, len = 0;
        bool clean = false;
        uint32_t rel = 0;
        if (valid) {
            s = off[r];
            len = off[r + 1] - s;
            rel = (uint32_t)(s - base);
            if (staged) {
                const LdsRead rv{reinterpret_cast<const uint32_t *>(stage), rel >> 2, rel & 3};
                clean = (read_flags(rv, (uint32_t)len) & 1) == 0;
            }
        }
        const uint32_t m = (clean && len >= (uint64_t)k) ? (uint32_t)(len - k + 1) : 0u;
        if (m) atomicMax(&s_rounds, (m + DS_R - 1) / DS_R);
        __syncthreads();
        const unsigned int nrounds = s_rounds;
        uint64_t fwd = 0, rc = 0;
        uint32_t t = 0, w = 0;
        if (m)
            for (; t < (uint32_t)(k - 1); t++) {
                const uint64_t b = code2(stage[rel + t]);
                fwd = ((fwd << 2) | b) & mask;
                rc = (rc >> 2) | ((3ull - b) << sh);
            }
        const uint32_t m2 = 2 * m - 1;
        for (unsigned int round = 0; round < nrounds; round++) {
            RecT rr[DS_R];
            unsigned int cb[DS_R], rk[DS_R];
#pragma unroll
            for (int j = 0; j < DS_R; j++) {
                cb[j] = 0xFFFFFFFFu;
                if (w < m) {
                    const uint64_t b = code2(stage[rel + t]);
                    fwd = ((fwd << 2) | b) & mask;
                    rc = (rc >> 2) | ((3ull - b) << sh);
                    rr[j] = make(fwd, rc, w, m2 - w, r, cb[j]);
                    rk[j] = atomicAdd(&bcnt[cb[j]], 1u);
                    t++;
                    w++;
                }
            }
            __syncthreads();
            // exclusive scan of the batch's bucket counts; reserve each bucket's run
            const unsigned int v = (int)tid < C ? bcnt[tid] : 0u;
            unsigned int incl = v;
            for (int o = 1; o < 64; o <<= 1) {
                const unsigned int u = __shfl_up(incl, o);
                if ((int)lane >= o) incl += u;
            }
            if (lane == 63) s_wave[wid] = incl;
            __syncthreads();
            unsigned int before = 0;
            for (unsigned int q = 0; q < wid; q++) before += s_wave[q];
            if ((int)tid < C) {
                bbeg[tid] = before + incl - v;
                gbase[tid] = cur[tid];
                cur[tid] += v;
            }
            if (tid == TILE_READS - 1) s_total = before + incl;
            __syncthreads();
#pragma unroll
            for (int j = 0; j < DS_R; j++) {
                if (cb[j] != 0xFFFFFFFFu) {
                    const unsigned int p = bbeg[cb[j]] + rk[j];
                    sorted[p] = rr[j];
                    sbk[p] = (uint8_t)cb[j];
                }
            }
            __syncthreads();
            const unsigned int total = s_total;
            for (unsigned int i = tid; i < total; i += TILE_READS) {
                const unsigned int c = sbk[i];
                recs.store(gbase[c] + (i - bbeg[c]), sorted[i]);
            }
            if ((int)tid < C) bcnt[tid] = 0;
            __syncthreads();
        }
        // reads with 'N' or an unstaged tile: reference-order slow path, direct stores
        if (valid && !clean) {
            auto slow = [&](auto &rd) {
                for_each_window(rd, s, len, k, r, [&](uint64_t f2, uint64_t r2, uint64_t ef, uint64_t er) {
                    unsigned int c;
                    const RecT rec = make(f2, r2, (uint32_t)ef, (uint32_t)er, r, c);
                    recs.store(atomicAdd(&cur[c], 1ull), rec);
                });
            };
            if (staged) {
                LdsReader lr{stage, base};
                slow(lr);
            } else {
                ByteReader br(buf);
                slow(br);
            }
        }
    }
}

// ---- refine: split each coarse bucket into its 2^(bbits-cbits) final buckets ----------------
// one workgroup per coarse bucket; tiles of REFINE_TILE records are sorted by final bucket in
// LDS and written out as contiguous runs (the final-bucket cursors live in LDS).
// gridDim.y workgroups share a coarse bucket (contiguous tile ranges); each tile reserves its
// runs in the final buckets with one global atomic per final bucket (cursor gcur, initialised
// to bstart).  Run order inside a final bucket is then arbitrary -- k_bucket is order-free.
// fcap != 0: the final buckets have a fixed capacity of fcap records from d * fcap (count_wide.h's
// third level, whose bucket sizes nothing counted): a record past its bucket's end is dropped
// and *over set (the caller then counts on the HBM table).
template <typename RecT, typename StoreIn, typename StoreOut>
__global__ void __launch_bounds__(BUCKET_THREADS) k_refine(StoreIn in, StoreOut out, const unsigned long long *bstart,
                                                          unsigned long long *gcur, int cbits, int bbits,
                                                          uint64_t fcap = 0, unsigned int *over = nullptr,
                                                          const unsigned long long *ibeg = nullptr,
                                                          const unsigned long long *iend = nullptr) {
    constexpr int TILE = sizeof(RecT) > 16 ? REFINE_TILE / 2 : REFINE_TILE;  // <= 64 KiB of LDS
    __shared__ RecT tile[TILE];
    __shared__ uint8_t tj[TILE];  // final bucket of each sorted record (the store loop needs no rehash)
    __shared__ unsigned long long base[REFINE_FANOUT];
    __shared__ unsigned int tcnt[REFINE_FANOUT], tbeg[REFINE_FANOUT], wsum[REFINE_FANOUT / 64];
    const int F = 1 << (bbits - cbits);
    const uint64_t c = blockIdx.x;
    // input: coarse bucket c's records [bstart[c F], bstart[(c + 1) F]), or [ibeg[c], iend[c])
    // when the coarse buckets are themselves fixed-capacity regions (join_w.h's levels)
    const uint64_t r0 = ibeg ? ibeg[c] : bstart[c * F], r1 = ibeg ? iend[c] : bstart[(c + 1) * F];
    const uint64_t nt = (r1 - r0 + TILE - 1) / TILE;
    const uint64_t tb = nt * blockIdx.y / gridDim.y, te = nt * (blockIdx.y + 1) / gridDim.y;
    constexpr int PER = TILE / BUCKET_THREADS;
    const uint64_t tend = min(r1, r0 + te * TILE);
    // software pipeline: tile t+1 is loaded into registers while tile t's runs are stored
    RecT nx[PER];
    auto load_tile = [&](uint64_t t0) {
        const unsigned int n = (unsigned int)min((uint64_t)TILE, r1 - t0);
#pragma unroll
        for (int q = 0; q < PER; q++) {
            const unsigned int i = threadIdx.x + q * BUCKET_THREADS;
            if (i < n) nx[q] = in.load(t0 + i);
        }
    };
    // (measured: pipelining pays for 12-B input, 4.86 -> 4.35 ms; 16-B input runs slower with it)
    constexpr bool PIPE = sizeof(RecT) < 16;
    uint64_t t0 = r0 + tb * TILE;
    if (t0 < tend) load_tile(t0);
    for (; t0 < tend; t0 += TILE) {
        if (!PIPE && t0 != r0 + tb * TILE) load_tile(t0);
        const unsigned int n = (unsigned int)min((uint64_t)TILE, r1 - t0);
        if (threadIdx.x < REFINE_FANOUT) tcnt[threadIdx.x] = 0;
        __syncthreads();
        RecT rr[PER];
        unsigned int jj[PER], rk[PER];
#pragma unroll
        for (int q = 0; q < PER; q++) {
            const unsigned int i = threadIdx.x + q * BUCKET_THREADS;
            rr[q] = nx[q];
            if (i < n) {
                jj[q] = rec_bucket(rr[q], bbits) & (F - 1);
                rk[q] = atomicAdd(&tcnt[jj[q]], 1u);
            }
        }
        __syncthreads();
        // exclusive scan of the tile counts + run reservation.  The reservation's returning
        // atomic is consumed only after the LDS scatter, so its latency overlaps the scatter
        // instead of stalling the whole workgroup at the next barrier.
        unsigned long long mybase = 0;
        if (threadIdx.x < REFINE_FANOUT) {
            const unsigned int v = (int)threadIdx.x < F ? tcnt[threadIdx.x] : 0u;
            unsigned int incl = v;
            for (int o = 1; o < 64; o <<= 1) {
                const unsigned int u = __shfl_up(incl, o);
                if ((int)(threadIdx.x & 63) >= o) incl += u;
            }
            tbeg[threadIdx.x] = incl - v;
            if ((threadIdx.x & 63) == 63) wsum[threadIdx.x >> 6] = incl;
            if (v) mybase = atomicAdd(&gcur[c * F + threadIdx.x], (unsigned long long)v);
        }
        __syncthreads();
        if (threadIdx.x >= 64 && threadIdx.x < REFINE_FANOUT) {
            unsigned int add = 0;
            for (unsigned int w = 0; w < (threadIdx.x >> 6); w++) add += wsum[w];
            tbeg[threadIdx.x] += add;
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < PER; q++) {
            const unsigned int i = threadIdx.x + q * BUCKET_THREADS;
            if (i < n) {
                const unsigned int p = tbeg[jj[q]] + rk[q];
                tile[p] = rr[q];
                tj[p] = (uint8_t)jj[q];
            }
        }
        if (threadIdx.x < REFINE_FANOUT) base[threadIdx.x] = mybase;
        __syncthreads();
        if (PIPE && t0 + TILE < tend) load_tile(t0 + TILE);
        if (fcap) {
            bool lost = false;
            for (unsigned int i = threadIdx.x; i < n; i += BUCKET_THREADS) {
                const unsigned int j = tj[i];
                const uint64_t pos = base[j] + (i - tbeg[j]);
                if (pos < (c * F + j + 1) * fcap) out.store(pos, tile[i]);
                else lost = true;
            }
            if (lost) *over = 1u;
        } else {
            for (unsigned int i = threadIdx.x; i < n; i += BUCKET_THREADS) {
                const unsigned int j = tj[i];
                out.store(base[j] + (i - tbeg[j]), tile[i]);
            }
        }
        __syncthreads();
    }
}

// ---- bucket counting in LDS -------------------------------------------------------------
// Structure of arrays, 32 B per slot.  (An array of 32-B slot structs put every key in one of
// four bank positions: a wave's 64 random probes then queued on a few banks -- PMC: 5.3·10^8
// LDS bank-conflict cycles in k_bucket.  Here consecutive slots' keys, counts and event pairs
// sit in consecutive banks.)
template <int SLOTS>
struct LTab {
    unsigned long long key[SLOTS];
    ulonglong2 ev[SLOTS];  // first events fC, fT: one ds_read_b128 reads both
    unsigned int count[SLOTS];
    unsigned int id[SLOTS];  // dense id carried by the records (DET sources)
};

// record sources of k_bucket: window records of the counting pass, or exchange records
// (count sum, first-event min) of the multi-GPU merge, visited through a bucket-major permutation
// Every source splits a record access into fetch (the loads) and decode (arithmetic), so
// k_bucket issues the loads of all its unrolled records before decoding any: a branch inside
// a decode (the even-k palindrome test) would otherwise serialise the loads behind it.
// Every source also has seg(b, y) (called before segment y of bucket b is read; k_bucket's
// buckets may be several record ranges), key_out(c) (the k-mer of table key c: sources whose
// table keys are not the k-mers themselves -- count_v2.h's hashed keys -- invert here) and
// slot_hash(c) (table placement: mix64, or the hashed key itself).
#define EC_PLAIN_SOURCE                                                              \
    __device__ inline void seg(uint32_t, uint32_t) {}                                \
    __device__ inline unsigned long long key_out(unsigned long long c) const { return c; } \
    __device__ inline uint64_t slot_hash(unsigned long long c) const { return mix64(c); }

struct RecSource {
    EC_PLAIN_SOURCE
    const Rec *recs;
    using Raw = Rec;
    static constexpr bool kDet = false;  // true: records carry their dense id (gathered solid set)
    __device__ inline Raw fetch(uint64_t i) const { return recs[i]; }
    __device__ inline unsigned int id(const Raw &) const { return 0; }
    __device__ inline void decode(const Raw &rec, unsigned long long &key, unsigned int &add, unsigned long long &eC,
                                  unsigned long long &eT) const {
        const unsigned int lC = rec.ev & 0xFFFFu, lT = rec.ev >> 16;
        key = rec.key;
        add = lC == lT ? 2u : 1u;  // even-k palindrome: build inserts it twice
        eC = ((unsigned long long)rec.read << 32) | lC;
        eT = ((unsigned long long)rec.read << 32) | lT;
    }
};

// compact record decode: meta = read << (ibits + 1) | orientation << ibits | window.  The
// even-k palindrome test is a template branch: left to a runtime k test the compiler evaluates
// twin64 for every record (k_bucket measured 45 % slower).
template <bool EVEN_K>
struct Rec12Decode {
    EC_PLAIN_SOURCE
    int ibits;
    int k;
    unsigned int m2;  // 2m - 1
    __device__ inline void decode(const Rec12 &r, unsigned long long &kk, unsigned int &add, unsigned long long &eC,
                                  unsigned long long &eT) const {
        kk = rkey(r);
        const unsigned int mt = r.meta;
        const unsigned long long rd = (unsigned long long)(mt >> (ibits + 1)) << 32;
        const unsigned int w = mt & ((1u << ibits) - 1), o = (mt >> ibits) & 1u;
        unsigned int lC = o ? m2 - w : w, lT = o ? w : m2 - w;
        add = 1;
        if (EVEN_K && twin64(kk, k) == kk) {  // even-k palindrome: inserted twice at the forward event
            add = 2;
            lC = lT = w;
        }
        eC = rd | lC;
        eT = rd | lT;
    }
};

template <bool EVEN_K>
struct Rec12Source : Rec12Decode<EVEN_K> {
    const unsigned long long *key;
    const unsigned int *meta;
    using Raw = Rec12;
    static constexpr bool kDet = false;
    __device__ inline unsigned int id(const Raw &) const { return 0; }
    __device__ inline Raw fetch(uint64_t i) const {
        const unsigned long long kk = key[i];
        Rec12 r;
        r.klo = (unsigned int)kk;
        r.khi = (unsigned int)(kk >> 32);
        r.meta = meta[i];
        return r;
    }
};

// packed 12-B records (Store12P: one array, dwordx3 accesses).  BIJ: the key words hold
// h = bij_fwd(key) (count_v2.h R10 path); the table counts h and key_out inverts it.
template <bool EVEN_K, bool BIJ = false>
struct Rec12PSource {
    int ibits;
    int k;
    unsigned int m2;  // 2m - 1
    const unsigned int *p;
    using Raw = Rec12;
    static constexpr bool kDet = false;
    __device__ inline void seg(uint32_t, uint32_t) {}
    __device__ inline unsigned long long key_out(unsigned long long c) const {
        return BIJ ? bij_inv(c, k, kmask64(k)) : c;
    }
    __device__ inline uint64_t slot_hash(unsigned long long c) const { return BIJ ? c : mix64(c); }
    __device__ inline unsigned int id(const Raw &) const { return 0; }
    __device__ inline Raw fetch(uint64_t i) const {
        Rec12 r;
        r.klo = p[3 * i];
        r.khi = p[3 * i + 1];
        r.meta = p[3 * i + 2];
        return r;
    }
    __device__ inline void decode(const Rec12 &r, unsigned long long &kk, unsigned int &add, unsigned long long &eC,
                                  unsigned long long &eT) const {
        kk = rkey(r);
        const unsigned int mt = r.meta;
        const unsigned long long rd = (unsigned long long)(mt >> (ibits + 1)) << 32;
        const unsigned int w = mt & ((1u << ibits) - 1), o = (mt >> ibits) & 1u;
        unsigned int lC = o ? m2 - w : w, lT = o ? w : m2 - w;
        add = 1;
        if (EVEN_K) {
            const unsigned long long x = key_out(kk);
            if (twin64(x, k) == x) {  // even-k palindrome: inserted twice at the forward event
                add = 2;
                lC = lT = w;
            }
        }
        eC = rd | lC;
        eT = rd | lT;
    }
};

// ---- LDS bucket table, shared by every bucket pass (window records, exchange records,
// super-k-mers): SLOTS open-addressing slots, CAS claim, count += add, atomicMin of events
// s_over[0] = overflow flag, s_over[1] = claimed slots.  A lane reserves a slot in the fill count
// before claiming one, and no claim takes the last free slot, so at least one slot stays empty
// and every probe sequence ends without a probe bound (a bounded loop costs the wave a
// counter, a compare and an exec-mask juggle per probe).
template <int SLOTS>
__device__ inline void lds_table_init(LTab<SLOTS> &tab, unsigned int *s_over) {
    for (int i = threadIdx.x; i < SLOTS; i += blockDim.x) {
        tab.key[i] = EMPTY_KEY;
        tab.count[i] = 0;
        tab.ev[i] = make_ulonglong2(NONE64, NONE64);
    }
    if (threadIdx.x == 0) {
        s_over[0] = 0;
        s_over[1] = 0;
    }
    __syncthreads();
}

// slot0 = first probe slot (the bucket sub-table's lookups start at the same slot).
// The probe loop is wave-uniform (runs while any lane still misses; lanes that found their
// slot idle under one exec mask): almost every wave has some lane past its first probe, and a
// per-lane loop with several exits costs ~40 scalar mask instructions per iteration.
// lds_locate: the slot of key c given its first probe (slot, cur = the key read there).
template <int SLOTS, typename Tab>
__device__ inline unsigned int lds_locate(Tab &tab, unsigned int *s_over, unsigned long long c,
                                          unsigned int slot, unsigned long long cur) {
    bool miss = cur != c;
#pragma unroll 1
    while (__any(miss)) {
        if (miss) {
            if (cur == EMPTY_KEY) {
                if (atomicAdd(&s_over[1], 1u) >= SLOTS - 1) {  // table full: the bucket is redone elsewhere
                    s_over[0] = 1;
                    cur = c;  // give up (updates below land in a discarded table)
                } else {
                    cur = atomicCAS(&tab.key[slot], EMPTY_KEY, c);
                    if (cur == EMPTY_KEY) cur = c;  // claimed
                    else atomicSub(&s_over[1], 1u);  // lost the race: cur = the winner's key
                }
            }
            if (cur != c) {
                slot = (slot + 1) & (SLOTS - 1);
                cur = tab.key[slot];
            }
            miss = cur != c;
        }
    }
    return slot;
}
// lds_locate of two keys at once (a lane's windows o and o + h): their probe chains run in one
// loop, so a step waits for the longer chain instead of the sum of both.
template <int SLOTS, typename Tab>
__device__ inline void lds_locate2(Tab &tab, unsigned int *s_over, unsigned long long cA, unsigned int &sA,
                                   unsigned long long curA, unsigned long long cB, unsigned int &sB,
                                   unsigned long long curB) {
    bool mA = curA != cA, mB = curB != cB;
    auto claim = [&](unsigned long long c, unsigned int slot, unsigned long long &cur) {
        if (atomicAdd(&s_over[1], 1u) >= SLOTS - 1) {  // table full: the bucket is redone elsewhere
            s_over[0] = 1;
            cur = c;
        } else {
            cur = atomicCAS(&tab.key[slot], EMPTY_KEY, c);
            if (cur == EMPTY_KEY) cur = c;
            else atomicSub(&s_over[1], 1u);
        }
    };
#pragma unroll 1
    while (__any(mA || mB)) {
        if (mA && curA == EMPTY_KEY) claim(cA, sA, curA);
        if (mB && curB == EMPTY_KEY) claim(cB, sB, curB);
        mA = curA != cA;
        mB = curB != cB;
        if (mA) sA = (sA + 1) & (SLOTS - 1);
        if (mB) sB = (sB + 1) & (SLOTS - 1);
        const unsigned long long nA = mA ? tab.key[sA] : cA, nB = mB ? tab.key[sB] : cB;
        curA = nA;
        curB = nB;
        mA = curA != cA;
        mB = curB != cB;
    }
}
template <int SLOTS, bool DET = false>
__device__ inline void lds_insert(LTab<SLOTS> &tab, unsigned int *s_over, unsigned long long c, unsigned int slot0,
                                  unsigned int add, unsigned long long eC, unsigned long long eT,
                                  unsigned int id = 0) {
    unsigned int slot = slot0 & (SLOTS - 1);
    slot = lds_locate<SLOTS>(tab, s_over, c, slot, tab.key[slot]);
    if (DET) tab.id[slot] = id;  // distinct keys: one writer per slot
    atomicAdd(&tab.count[slot], add);
    const ulonglong2 ev = tab.ev[slot];
    if (eC < ev.x) atomicMin(&tab.ev[slot].x, eC);
    if (eT < ev.y) atomicMin(&tab.ev[slot].y, eT);
}

// solid filter (count > limit, build:37-39) + compaction of bucket b's table into the dense
// arrays (wave ballot, one global atomic per block) + the bucket's lookup sub-table
struct KeyId {
    __device__ inline unsigned long long operator()(unsigned long long c) const { return c; }
};
// the first events of slot i as stored (LTab: (read << 32) | l per orientation)
struct EvId {
    template <typename Tab>
    __device__ inline ulonglong2 operator()(const Tab &tab, int i) const { return tab.ev[i]; }
};
template <int SLOTS, bool DET = false, typename KO = KeyId, typename Tab = LTab<SLOTS>, typename EO = EvId,
          int NT = BUCKET_THREADS>
__device__ inline void lds_table_finish(const Tab &tab, const unsigned int *s_over, unsigned int b,
                                        long long limit,
                                        unsigned long long *dkey, unsigned int *dcnt, unsigned long long *dfc,
                                        unsigned long long *dft, SubSlot *sub, unsigned int *nsolid,
                                        unsigned long long *ndistinct, unsigned int *overflow, KO ko = KO(),
                                        EO eo = EO(), unsigned int *bmark = nullptr) {
    __shared__ unsigned int s_wave[NT / 64], s_pres[NT / 64];
    __shared__ unsigned int s_base;
    __syncthreads();
    if (*s_over) {
        if (threadIdx.x == 0) atomicAdd(overflow, 1u);
        return;
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    constexpr int PER = SLOTS / NT;
    if constexpr (DET) {  // dense ids given by the records (LTab::id): every present key is solid
        SubSlot *region = sub + (uint64_t)b * SLOTS;
        for (int q = 0; q < PER; q++) {
            const int i = threadIdx.x * PER + q;
            const unsigned long long key = tab.key[i];
            SubSlot o;
            o.key = key;
            o.id = NONE32;
            o.pad = 0;
            if (key != EMPTY_KEY) {
                const unsigned int u = tab.id[i];
                const ulonglong2 ev = eo(tab, i);
                dkey[u] = ko(key);
                dcnt[u] = tab.count[i];
                dfc[u] = ev.x;
                dft[u] = ev.y;
                o.id = u;
            }
            region[i] = o;
        }
        return;
    }
    bool solid[PER];
    unsigned int mine = 0, present = 0;
    for (int q = 0; q < PER; q++) {
        const int i = threadIdx.x * PER + q;
        const bool here = tab.key[i] != EMPTY_KEY;
        present += here;
        solid[q] = here && (long long)tab.count[i] > limit;
        mine += solid[q];
    }
    // wave exclusive scan of `mine`
    unsigned int incl = mine;
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned int v = __shfl_up(incl, o);
        if (lane >= o) incl += v;
    }
    if (lane == 63) s_wave[wid] = incl;
    unsigned int pres = present;
    for (int o = 32; o > 0; o >>= 1) pres += __shfl_down(pres, o);
    if (lane == 0) s_pres[wid] = pres;
    __syncthreads();
    if (threadIdx.x == 0) {  // one global atomic each per block (a per-wave atomic on one word serialises)
        unsigned int tot = 0, np = 0;
        for (int w = 0; w < NT / 64; w++) {
            const unsigned int c = s_wave[w];
            s_wave[w] = tot;
            tot += c;
            np += s_pres[w];
        }
        s_base = tot ? atomicAdd(nsolid, tot) : 0;
        if (bmark && tot) atomicOr(&bmark[s_base >> 5], 1u << (s_base & 31));  // (the bucket's first id: k_tile_plan)
        if (np && ndistinct) atomicAdd(ndistinct, (unsigned long long)np);
    }
    __syncthreads();
    unsigned int u = s_base + s_wave[wid] + incl - mine;
    SubSlot *region = sub + (uint64_t)b * SLOTS;
    for (int q = 0; q < PER; q++) {
        const int i = threadIdx.x * PER + q;
        SubSlot o;
        o.key = tab.key[i];
        o.id = NONE32;
        o.pad = 0;
        if (solid[q]) {
            const ulonglong2 ev = eo(tab, i);
            dkey[u] = ko(o.key);
            dcnt[u] = tab.count[i];
            dfc[u] = ev.x;
            dft[u] = ev.y;
            o.id = u;
            u++;
        }
        if (sub) region[i] = o;  // no lookup index wanted (shard counts, owner merges): skip the dump
    }
}

// the k-mer of a table key for the dense arrays (count_v2.h hashed keys are inverted)
template <typename Src>
struct KeyOutOf {
    Src src;
    __device__ inline unsigned long long operator()(unsigned long long c) const { return src.key_out(c); }
};

// bucket b = record ranges [bbeg[b * nseg + y], bend[b * nseg + y]) for y < nseg
template <typename Src, int SLOTS>
__global__ void __launch_bounds__(BUCKET_THREADS) k_bucket(Src src, const unsigned long long *bbeg,
                                                          const unsigned long long *bend, uint32_t nseg,
                                                          long long limit,
                                                          unsigned long long *dkey, unsigned int *dcnt,
                                                          unsigned long long *dfc, unsigned long long *dft,
                                                          SubSlot *sub, unsigned int *nsolid,
                                                          unsigned long long *ndistinct, unsigned int *overflow,
                                                          unsigned int *bmark = nullptr) {
    __shared__ LTab<SLOTS> tab;
    __shared__ unsigned int s_over[2];
    const unsigned int b = blockIdx.x;
    lds_table_init<SLOTS>(tab, s_over);
    // BK_UNROLL records per thread per step, all loads issued before the inserts: the loop
    // is bound by HBM latency, not bandwidth, without this memory-level parallelism
    constexpr int BK_UNROLL = 4;
    for (uint32_t y = 0; y < nseg; y++) {
        Src s = src;
        s.seg(b, y);
        const uint64_t r0 = bbeg[(uint64_t)b * nseg + y], r1 = bend[(uint64_t)b * nseg + y];
        uint64_t i = r0 + threadIdx.x;
        for (; i + (BK_UNROLL - 1) * (uint64_t)blockDim.x < r1; i += BK_UNROLL * (uint64_t)blockDim.x) {
            typename Src::Raw raw[BK_UNROLL];
#pragma unroll
            for (int u = 0; u < BK_UNROLL; u++) raw[u] = s.fetch(i + u * (uint64_t)blockDim.x);
#pragma unroll
            for (int u = 0; u < BK_UNROLL; u++) {
                unsigned long long c, eC, eT;
                unsigned int add;
                s.decode(raw[u], c, add, eC, eT);
                lds_insert<SLOTS, Src::kDet>(tab, s_over, c, (unsigned int)s.slot_hash(c), add, eC, eT, s.id(raw[u]));
            }
        }
        for (; i < r1; i += blockDim.x) {
            unsigned long long c, eC, eT;
            unsigned int add;
            const typename Src::Raw r = s.fetch(i);
            s.decode(r, c, add, eC, eT);
            lds_insert<SLOTS, Src::kDet>(tab, s_over, c, (unsigned int)s.slot_hash(c), add, eC, eT, s.id(r));
        }
    }
    lds_table_finish<SLOTS, Src::kDet>(tab, s_over, b, limit, dkey, dcnt, dfc, dft, sub, nsolid, ndistinct,
                                       overflow, KeyOutOf<Src>{src}, EvId(), bmark);
}

// ---- buckets with more distinct k-mers than an LDS table holds -----------------------------
// Two cases: error-rich inputs (most distinct k-mers occur once: 150 M distinct for 4.6 M solid
// at 0.5 % substitutions, 10 M x 100 bp) and large genomes (> ~2·10^7 solid k-mers).  A key
// occurring once is solid only if its single insert adds more than `limit` (an even-k
// palindrome adds 2), so with limit >= 1 the workgroup first builds a "seen twice" filter over
// the bucket's records (two 2^18-cell bitmaps: cell bit set on the second sighting, two cells
// per key -- no false negatives, ~2 % of the singletons leak).  From the bitmap it estimates
// the keys it will insert (linear counting over the set cells) and splits the bucket into
// 2^pb parts by hash bits 11.. (pb <= pmax), one table pass each; part q's table becomes
// sub-table region (b << pmax) + q, and bnp[b] = pb tells the lookup how the bucket was split
// (SolidIndex::npb).  With limit < 1 (the multi-GPU shard count: singletons may meet their
// twins on other ranks) every key is kept; the bitmap then only counts the distinct keys.
constexpr int FILT_BITS = 18;
constexpr double PART_KEYS = 1400.0;  // target keys per 2048-slot part table
template <typename Src>
__global__ void __launch_bounds__(BUCKET_THREADS) k_bucket_filt(Src src, const unsigned long long *bbeg,
                                                               const unsigned long long *bend, uint32_t nseg,
                                                               long long limit, int pmin, int pmax, float part_keys,
                                                               unsigned long long *dkey,
                                                               unsigned int *dcnt, unsigned long long *dfc,
                                                               unsigned long long *dft, SubSlot *sub, uint8_t *bnp,
                                                               unsigned int *nsolid, unsigned long long *ndistinct,
                                                               unsigned int *overflow) {
    constexpr int SLOTS = 2048;
    constexpr unsigned int NW = 1u << (FILT_BITS - 5);
    constexpr unsigned int CM = (1u << FILT_BITS) - 1;
    __shared__ LTab<SLOTS> tab;
    __shared__ unsigned int s_over[2];
    __shared__ unsigned int seen1[NW], seen2[NW];
    __shared__ unsigned int s_cells, s_pb;
    const unsigned int b = blockIdx.x;
    for (unsigned int i = threadIdx.x; i < NW; i += blockDim.x) {
        seen1[i] = 0;
        seen2[i] = 0;
    }
    if (threadIdx.x == 0) s_cells = 0;
    __syncthreads();
    constexpr int U = 4;  // records per thread per step, loads issued before any decode
    auto for_records = [&](auto &&fn) {
        for (uint32_t y = 0; y < nseg; y++) {
            Src s = src;
            s.seg(b, y);
            const uint64_t r0 = bbeg[(uint64_t)b * nseg + y], r1 = bend[(uint64_t)b * nseg + y];
            uint64_t i = r0 + threadIdx.x;
            for (; i + (U - 1) * (uint64_t)blockDim.x < r1; i += U * (uint64_t)blockDim.x) {
                typename Src::Raw raw[U];
#pragma unroll
                for (int u = 0; u < U; u++) raw[u] = s.fetch(i + u * (uint64_t)blockDim.x);
#pragma unroll
                for (int u = 0; u < U; u++) fn(s, raw[u]);
            }
            for (; i < r1; i += blockDim.x) fn(s, s.fetch(i));
        }
    };
    // pass 0: seen-twice filter (limit >= 1) or distinct-key bitmap (limit < 1)
    const bool filter = limit >= 1;
    for_records([&](const Src &s, const typename Src::Raw &r) {
        unsigned long long c, eC, eT;
        unsigned int add;
        s.decode(r, c, add, eC, eT);
        const uint64_t h = mix64(c);  // filter cells (the part tables follow slot_hash)
        const unsigned int c1 = (unsigned int)(h >> 12) & CM, c2 = (unsigned int)(h >> 30) & CM;
        const unsigned int m1 = 1u << (c1 & 31), m2 = 1u << (c2 & 31);
        if (filter) {
            if (atomicOr(&seen1[c1 >> 5], m1) & m1) atomicOr(&seen2[c1 >> 5], m1);
            if (atomicOr(&seen1[c2 >> 5], m2) & m2) atomicOr(&seen2[c2 >> 5], m2);
        } else if (!(seen1[c1 >> 5] & m1)) {
            atomicOr(&seen1[c1 >> 5], m1);
        }
    });
    __syncthreads();
    // keys to insert, by linear counting over the cells (filter: two cells per key); with the
    // filter, the bucket's distinct keys (filtered singletons included) by the same estimate over
    // the seen-once cells -- ndistinct is then an estimate (+-2 %), exact otherwise
    __shared__ unsigned int s_cells1;
    {
        if (threadIdx.x == 0) s_cells1 = 0;
        unsigned int cells = 0, cells1 = 0;
        const unsigned int *w = filter ? seen2 : seen1;
        for (unsigned int i = threadIdx.x; i < NW; i += blockDim.x) {
            cells += __popc(w[i]);
            cells1 += __popc(seen1[i]);
        }
        for (int o = 32; o > 0; o >>= 1) {
            cells += __shfl_down(cells, o);
            cells1 += __shfl_down(cells1, o);
        }
        __syncthreads();
        if ((threadIdx.x & 63) == 0) {
            atomicAdd(&s_cells, cells);
            atomicAdd(&s_cells1, cells1);
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            const double m = (double)(1u << FILT_BITS), set = (double)min(s_cells, (1u << FILT_BITS) - 1);
            const double keys = -m * log(1.0 - set / m) / (filter ? 2.0 : 1.0);
            unsigned int pb = (unsigned int)pmin;  // (pmin > 0: tests force the split)
            while ((int)pb < pmax && keys / (double)(1u << pb) > (double)part_keys) pb++;
            // more keys than even the 2^pmax part tables hold (2047 each; 10 % above the linear-
            // counting error): report the overflow now instead of after all the table passes
            if (keys / (double)(1u << pb) > 2047.0 * 1.1) pb = 0xFFu;
            s_pb = pb;
            if (bnp && pb != 0xFFu) bnp[b] = (uint8_t)pb;
            if (filter && pb != 0xFFu) {
                const double set1 = (double)min(s_cells1, (1u << FILT_BITS) - 1);
                atomicAdd(ndistinct, (unsigned long long)llround(-m * log(1.0 - set1 / m) / 2.0));
            }
        }
        __syncthreads();
    }
    if (s_pb == 0xFFu) {
        if (threadIdx.x == 0) atomicAdd(overflow, 1u);
        return;
    }
    const unsigned int pb = s_pb, pmask = (1u << pb) - 1;
    for (unsigned int part = 0; part <= pmask; part++) {
        lds_table_init<SLOTS>(tab, s_over);
        for_records([&](const Src &s, const typename Src::Raw &r) {
            unsigned long long c, eC, eT;
            unsigned int add;
            s.decode(r, c, add, eC, eT);
            const uint64_t hs = s.slot_hash(c), h = mix64(c);
            if (((unsigned int)(hs >> 11) & pmask) != part) return;
            if (filter) {
                const unsigned int c1 = (unsigned int)(h >> 12) & CM, c2 = (unsigned int)(h >> 30) & CM;
                const bool twice = ((seen2[c1 >> 5] >> (c1 & 31)) & (seen2[c2 >> 5] >> (c2 & 31)) & 1u) != 0;
                if (!twice && (long long)add <= limit) return;
            }
            lds_insert<SLOTS>(tab, s_over, c, (unsigned int)hs, add, eC, eT);
        });
        lds_table_finish<SLOTS>(tab, s_over, (b << pmax) + part, limit, dkey, dcnt, dfc, dft, sub, nsolid,
                                filter ? nullptr : ndistinct, overflow, KeyOutOf<Src>{src});
        __syncthreads();
        if (s_over[0]) break;  // overflow already reported: the call is redone on the HBM table
    }
}

}  // namespace ec
