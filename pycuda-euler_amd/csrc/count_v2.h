// count_v2.h -- partitioned k-mer counting without the histogram upsweep (the default path of
// build:25-42 for N-free reads of one length, k <= 32).
//
// count_part.h sizes every (coarse bucket, read group) run exactly from a per-window fine
// histogram (k_upsweep: every window hashed and counted once more before the downsweep).  Here
// the runs get a fixed capacity instead -- the placement hash is uniform, so a group's records
// per coarse bucket stay within a few standard deviations of (its windows) / C -- and the pass
// before the downsweep only has to read bytes:
//
//   k_prescan    per read group : SWAR alphabet / N check of the group's bytes, read lengths,
//                                 windows (no hashing)
//   k_partition  per read group : each WAVE independently stages 64 reads in its own LDS
//                                 slice (the next tile's loads in flight in registers while it
//                                 works), rolls 8 windows per lane per round, ranks them by
//                                 coarse bucket with LDS atomics on its own counters, and
//                                 stores bucket runs; a run of the (bucket, group) region is
//                                 reserved by one LDS atomic on the workgroup cursor.  No
//                                 workgroup barrier inside the loop.  Also the HyperLogLog
//                                 registers (the distinct estimate sets the bucket count).
//   k_refine2    per coarse bucket slice : the region runs -> final buckets of fixed capacity
//                                 (packed 12-B records, one returning atomic per final bucket
//                                 per tile)
//   k_bucket     (count_part.h) per final bucket, unchanged
//
// Any run or final bucket past its capacity (extreme k-mer skew) is reported, and the call
// is redone on count_part.h's exact path.
#pragma once
#include "count_part.h"

namespace ec {

constexpr int PT_WAVES = 4;                // waves per k_partition workgroup
constexpr int PT_THREADS = 64 * PT_WAVES;
#ifndef PT_W_DEF
#define PT_W_DEF 8
#endif
constexpr int PT_W = PT_W_DEF;             // windows per lane per round
constexpr int PT_REC = 64 * PT_W;          // records per wave round
constexpr int PT_CBITS = 5;                // coarse buckets (one lane each)
constexpr int PT_MAX_NPF = 8;              // staged bytes per wave tile <= PT_MAX_NPF KiB

// wave-scope ordering of LDS accesses between the lanes of one wave (LDS operations of a wave
// execute in issue order; this only keeps the compiler from moving them across)
__device__ inline void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// inclusive prefix sum over the 64 lanes of a wave (DPP row shifts + row broadcasts)
__device__ inline unsigned int wave_incl_scan(unsigned int v) {
    v += (unsigned int)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);  // row_shr:1
    v += (unsigned int)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);  // row_shr:2
    v += (unsigned int)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);  // row_shr:4
    v += (unsigned int)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);  // row_shr:8
    v += (unsigned int)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15
    v += (unsigned int)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);  // row_bcast:31
    return v;
}

// 0x80 in every zero byte of v, 0 elsewhere (exact per byte: no borrow between bytes)
__device__ inline uint32_t zero_bytes(uint32_t v) {
    return ~(((v & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | v | 0x7F7F7F7Fu);
}
// 0x80 in every byte of w that is A, C, G or T
__device__ inline uint32_t acgt_bytes(uint32_t w) {
    return zero_bytes(w ^ 0x41414141u) | zero_bytes(w ^ 0x43434343u) | zero_bytes(w ^ 0x47474747u) |
           zero_bytes(w ^ 0x54545454u);
}

// ---- prescan: alphabet, N, lengths, windows per read group ---------------------------------
// lens[0] = max length of reads with windows, lens[1] = ~min of those, lens[2] = some read
// holds an 'N', lens[3] = max length of any read; *bad = first byte outside {A,C,G,T,N}
__global__ void __launch_bounds__(256) k_prescan(const uint8_t *buf, const uint64_t *off, uint64_t nreads, int k,
                                                 uint64_t gsize, unsigned long long *npos, unsigned long long *bad,
                                                 unsigned int *lens) {
    const uint64_t g = blockIdx.x;
    const uint64_t g0 = min(g * gsize, nreads), g1 = min(g0 + gsize, nreads);
    unsigned long long pos = 0;
    unsigned int lmax = 0, lmin = 0xFFFFFFFFu, lall = 0, anyn = 0;
    auto length = [&](uint64_t len) {
        lall = max(lall, (unsigned int)min(len, (uint64_t)0xFFFFFFFFu));
        if (len >= (uint64_t)k) {
            lmax = max(lmax, (unsigned int)min(len, (uint64_t)0xFFFFFFFFu));
            lmin = min(lmin, (unsigned int)min(len, (uint64_t)0xFFFFFFFFu));
            pos += len - k + 1;
        }
    };
    {  // read lengths, four offset pairs per thread in flight
        uint64_t r = g0 + threadIdx.x;
        for (; r + 3 * blockDim.x < g1; r += 4 * blockDim.x) {
            uint64_t a[4], b[4];
#pragma unroll
            for (int u = 0; u < 4; u++) a[u] = off[r + u * blockDim.x], b[u] = off[r + u * blockDim.x + 1];
#pragma unroll
            for (int u = 0; u < 4; u++) length(b[u] - a[u]);
        }
        for (; r < g1; r += blockDim.x) length(off[r + 1] - off[r]);
    }
    if (g1 > g0) {
        const uint64_t b0 = off[g0], b1 = off[g1];
        const uint64_t a0 = ((uint64_t)(buf + b0)) & ~15ull, a1 = (((uint64_t)(buf + b1)) + 15) & ~15ull;
        const uint64_t n16 = (a1 - a0) >> 4, lo = (uint64_t)buf + b0, hi = (uint64_t)buf + b1;
        const uint4 *src = reinterpret_cast<const uint4 *>(buf + b0 - (((uint64_t)(buf + b0)) & 15));
        auto check = [&](const uint4 &v, uint64_t i) {
            const uint64_t a = a0 + 16 * i;
            uint32_t all = acgt_bytes(v.x) & acgt_bytes(v.y) & acgt_bytes(v.z) & acgt_bytes(v.w);
            if (a < lo || a + 16 > hi) all = 0;  // partial chunk: byte by byte
            if (all != 0x80808080u) {
                const uint32_t w[4] = {v.x, v.y, v.z, v.w};
                for (int q = 0; q < 16; q++) {
                    const uint64_t p = a + q;
                    if (p < lo || p >= hi) continue;
                    const uint32_t c = base_code((w[q >> 2] >> ((q & 3) * 8)) & 0xFFu);
                    if (c == 4) anyn = 1;
                    if (c == 5) atomicMin(bad, (unsigned long long)(p - (uint64_t)buf));
                }
            }
        };
        // eight 16-B loads per thread in flight before any check
        constexpr int U = 8;
        uint64_t i = threadIdx.x;
        for (; i + (U - 1) * blockDim.x < n16; i += U * blockDim.x) {
            uint4 v[U];
#pragma unroll
            for (int u = 0; u < U; u++) v[u] = src[i + u * blockDim.x];
#pragma unroll
            for (int u = 0; u < U; u++) check(v[u], i + u * blockDim.x);
        }
        for (; i < n16; i += blockDim.x) check(src[i], i);
    }
    for (int o = 32; o > 0; o >>= 1) {
        pos += __shfl_down(pos, o);
        lmax = max(lmax, (unsigned int)__shfl_down(lmax, o));
        lmin = min(lmin, (unsigned int)__shfl_down(lmin, o));
        lall = max(lall, (unsigned int)__shfl_down(lall, o));
        anyn |= (unsigned int)__shfl_down(anyn, o);
    }
    // one set of global atomics per workgroup (per wave they queued on the same five words)
    __shared__ unsigned long long s_pos[4];
    __shared__ unsigned int s_l[4][4];
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        s_pos[w] = pos;
        s_l[w][0] = lmax, s_l[w][1] = lmin, s_l[w][2] = anyn, s_l[w][3] = lall;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int q = 1; q < (int)(blockDim.x >> 6); q++) {
            pos += s_pos[q];
            lmax = max(lmax, s_l[q][0]), lmin = min(lmin, s_l[q][1]), anyn |= s_l[q][2], lall = max(lall, s_l[q][3]);
        }
        if (pos) atomicAdd(npos, pos);
        if (lmax) atomicMax(&lens[0], lmax);
        if (lmin != 0xFFFFFFFFu) atomicMax(&lens[1], ~lmin);
        if (anyn) atomicOr(&lens[2], 1u);
        if (lall) atomicMax(&lens[3], lall);
    }
}

// ---- partition: window records into fixed-capacity (coarse bucket, group) runs ------------
// 4 ASCII bases (A C G T) -> 8 bits, base i at bits 2i (code2 of window.h, no table)
__device__ inline uint32_t pack4(uint32_t w) {
    const uint32_t x = ((w >> 1) ^ (w >> 2)) & 0x03030303u;
    const uint32_t y = x | (x >> 6);
    return (y | (y >> 12)) & 0xFFu;
}
__device__ inline uint32_t pack16(const uint4 &v) {
    return pack4(v.x) | (pack4(v.y) << 8) | (pack4(v.z) << 16) | (pack4(v.w) << 24);
}

// Next wave tile's bytes into pf[] and its reads' offsets (k_partition, k_skpart): uses the
// kernel's g0, g1, off, buf, lane, pf, nx_base, nx_s, nx_e, nx_n; nx_lo / nx_hi = the tile's
// read bytes relative to nx_base, nx_n16 = its 16-B chunks
// (a macro, not a lambda: a lambda capturing pf keeps the array in scratch memory)
#define EC_PT_ISSUE(T)                                                                                   \
    do {                                                                                                 \
        const uint64_t r0_ = g0 + 64ull * (T), r1_ = min(r0_ + 64, g1);                                  \
        const uint64_t b0_ = off[r0_], b1_ = off[r1_]; /* wave-uniform: scalar loads */                  \
        const uint8_t *p0_ = buf + b0_ - (((uint64_t)(buf + b0_)) & 15); /* derived from buf: global */  \
        const uint64_t a1_ = (((uint64_t)(buf + b1_)) + 15) & ~15ull;                                      \
        const uint32_t n16_ = (uint32_t)((a1_ - (uint64_t)p0_) >> 4); /* <= NPF * 64: host checks */    \
        const uint4 *src_ = reinterpret_cast<const uint4 *>(p0_);                                         \
        _Pragma("unroll") for (int q = 0; q < NPF; q++)                                                   \
            pf[q] = src_[min(q * 64 + lane, n16_ - 1)]; /* in bounds: no branch around the load */       \
        nx_base = (uint64_t)p0_ - (uint64_t)buf;                                                         \
        nx_lo = (uint32_t)(b0_ - nx_base), nx_hi = (uint32_t)(b1_ - nx_base), nx_n16 = n16_;             \
        /* low words of the read's offsets (differences mod 2^32; no wait until they are used) */       \
        const uint64_t ri_ = min(r0_ + lane, r1_ - 1);                                                   \
        nx_s = reinterpret_cast<const uint32_t *>(off)[2 * ri_];                                         \
        nx_e = reinterpret_cast<const uint32_t *>(off)[2 * ri_ + 2];                                     \
        nx_n = (uint32_t)(r1_ - r0_);                                                                    \
    } while (0)

// Every read with windows has exactly M windows and no N (k_prescan checked).  Record of
// window w of read r: key = canonical code, meta = (read_base + r) << (ibits + 1) | o << ibits | w
// (Rec12, count_part.h).  Region of (c, g): records [(g * C + c) * cap, + cap) of keys / meta
// (group-major: the C regions a workgroup appends to are adjacent, so its stores stay within a
// few pages of address translation; coarse-bucket-major spread them 2 GiB and missed UTCL1);
// records [C * G * cap, + PT_REC) take the stores of a run past its capacity (*overflow is set
// and the call is redone on the exact path).  cnt[c * G + g] = records stored in the region.
// HyperLogLog over the keys whose low hash bits & smask are 0 (a 1 / (smask + 1) sample of the
// key space): hll[g * 2^HLL_REG_BITS + j] = the group's register j.
// The wave tile's bytes are staged 2 bits per base (word i = bases 16i .. 16i+15 of the tile).
//
// R10 (10-byte records, Pack10): the key is placed by h = bij_fwd(key) (coarse bucket = its top
// PT_CBITS bits) and the record keeps the remnant h mod 2^(2k - PT_CBITS) and a group-relative
// meta (read - g0 << (ibits + 1) | o << ibits | w); `meta` is then a uint16_t array.
template <int NPF, bool HI, bool R10>
__global__ void __launch_bounds__(PT_THREADS) k_partition(const uint8_t *__restrict__ buf,
                                                          const uint64_t *__restrict__ off, uint64_t nreads,
                                                          int k, uint32_t M, uint64_t gsize, uint32_t G, uint64_t cap,
                                                          int ibits, uint64_t read_base, uint32_t smask,
                                                          unsigned long long *keys, void *metap,
                                                          unsigned int *cnt, uint8_t *hll, unsigned int *overflow) {
    constexpr int C = 1 << PT_CBITS;
    constexpr int NREG = 1 << HLL_REG_BITS;
    constexpr int SW = NPF * 64 + 4;  // staged words per wave (+ reads past the last base)
    __shared__ uint32_t s_stage[PT_WAVES][SW];
    __shared__ unsigned long long s_key[PT_WAVES][PT_REC + 1];  // + a dummy slot for invalid windows
    __shared__ unsigned int s_meta[PT_WAVES][PT_REC + 1];
    __shared__ uint8_t s_tag[PT_WAVES][PT_REC + 1];
    __shared__ unsigned long long s_base[PT_WAVES][C];  // store index of sorted record 0 of bucket c
    __shared__ unsigned int s_wcnt[PT_WAVES][C + 1];    // + a dummy counter
    __shared__ unsigned int s_cur[C];
    __shared__ unsigned int s_hll[NREG / 4];  // u8 registers, four per word
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // uniform: scalar tile loads
    for (int i = threadIdx.x; i < NREG / 4; i += PT_THREADS) s_hll[i] = 0;
    if (threadIdx.x < C) s_cur[threadIdx.x] = 0;
    if (lane <= C) s_wcnt[wid][lane] = 0;
    __syncthreads();
    const uint64_t g = blockIdx.x;
    const uint64_t g0 = min(g * gsize, nreads), g1 = min(g0 + gsize, nreads);
    const uint32_t ntile = (uint32_t)((g1 - g0 + 63) / 64);
    const uint64_t mask = kmask64(k);
    const uint32_t mhi = (uint32_t)(mask >> 32);
    const int sh = 2 * (k - 1);
    uint64_t fwd = 0, rc = 0;
    auto roll = [&](uint32_t b) {
        if (HI) {
            fwd = (fwd << 2) | b;
            fwd &= ((uint64_t)mhi << 32) | 0xFFFFFFFFull;
            rc = (rc >> 2) | ((uint64_t)((3u - b) << (sh - 32)) << 32);
        } else {
            fwd = ((fwd << 2) | b) & mask;
            rc = (rc >> 2) | ((uint64_t)(3u - b) << sh);
        }
    };
    // the next tile's bytes (in flight while the current tile is processed) and its reads
    uint4 pf[NPF];
    uint64_t nx_base = 0;
    uint32_t nx_s = 0, nx_e = 0, nx_n = 0, nx_lo = 0, nx_hi = 0, nx_n16 = 0;
    (void)nx_lo;
    if (wid < ntile) EC_PT_ISSUE(wid);
    const unsigned long long gcap = g * C * cap, gstride = cap;
    const unsigned long long spill = (unsigned long long)C * G * cap;
    const uint32_t mbits = ibits + 1;
    const int rb = 2 * k - PT_CBITS;  // R10: remnant bits
    const uint64_t rmask = rb >= 64 ? ~0ull : (1ull << rb) - 1;
    uint32_t *st = s_stage[wid];
    for (uint32_t t = wid; t < ntile; t += PT_WAVES) {
        // stage this tile 2 bits per base, then put the next one in flight
#pragma unroll
        for (int q = 0; q < NPF; q++) st[q * 64 + lane] = pack16(pf[q]);
        const uint32_t tbase = (uint32_t)nx_base, s = nx_s;
        const uint32_t len = lane < nx_n ? nx_e - nx_s : 0u;
        const uint64_t r = g0 + 64ull * t + lane;
        const bool more = t + PT_WAVES < ntile;
        wave_sync();
        const bool has = len >= (uint32_t)k;  // then len - k + 1 == M
        const uint32_t rel = has ? s - tbase : 0u;  // the read's first base in the tile
        const uint32_t mhead = R10 ? (uint32_t)((r - g0) << mbits) : (uint32_t)((r + read_base) << mbits);
        // bases p .. p + 15 of the tile, base p + i at bits 2i
        auto bases16 = [&](uint32_t p) { return __builtin_amdgcn_alignbit(st[(p >> 4) + 1], st[p >> 4], 2 * (p & 15)); };
        fwd = 0;
        rc = 0;
        {
            const uint32_t x0 = bases16(rel), x1 = bases16(rel + 16);
            for (uint32_t tb = 0; tb < (uint32_t)(k - 1); tb++)
                roll(tb < 16 ? (x0 >> (2 * tb)) & 3u : (x1 >> (2 * (tb - 16))) & 3u);
        }
        const uint32_t nrounds = __any(has) ? (M + PT_W - 1) / PT_W : 0u;
        if (nrounds == 0 && more) EC_PT_ISSUE(t + PT_WAVES);
        uint32_t w = 0, tb = (uint32_t)(k - 1);
        for (uint32_t round = 0; round < nrounds; round++, tb += PT_W) {
            const uint32_t xb = bases16(rel + tb);
            unsigned long long rkey[PT_W];
            unsigned int rmeta[PT_W], rcb[PT_W], rhh[PT_W];
            unsigned int smp = 0;  // windows whose key is in the HyperLogLog sample
#pragma unroll
            for (int j = 0; j < PT_W; j++) {
                roll((xb >> (2 * j)) & 3u);
                const bool tw = fwd > rc;
                const uint64_t c = tw ? rc : fwd;
                const bool ok = has && w + j < M;
                const uint32_t mt = mhead | ((tw ? 1u : 0u) << ibits) | (w + j);
                uint64_t h;
                uint32_t hh;  // 32 well-mixed hash bits: the bucket in the top PT_CBITS
                if (R10) {
                    h = bij_fwd(c, k, mask);
                    hh = (uint32_t)((h << (64 - 2 * k)) >> 32);
                    rkey[j] = (h & rmask) | ((uint64_t)(mt >> 16) << rb);
                    rmeta[j] = mt & 0xFFFFu;
                } else {
                    h = mix64(c);
                    hh = (uint32_t)(h >> 32);
                    rkey[j] = c;
                    rmeta[j] = mt;
                }
                rcb[j] = ok ? hh >> (32 - PT_CBITS) : (uint32_t)C;  // C: a dummy counter
                rhh[j] = hh;
                smp |= (ok && ((uint32_t)h & smask) == 0) ? 1u << j : 0u;
                atomicAdd(&s_wcnt[wid][rcb[j]], 1u);  // bucket sizes (no return value)
            }
            w += PT_W;
            // the next tile's loads go out in the last round (their wait at the next tile then
            // does not also wait for a whole tile of stores)
            if (round + 1 == nrounds && more) EC_PT_ISSUE(t + PT_WAVES);
            // HyperLogLog registers (count_part.h k_upsweep's rho), u8 max by CAS
            if (__any(smp)) {
#pragma unroll
                for (int j = 0; j < PT_W; j++) {
                    if (!((smp >> j) & 1u)) continue;
                    const uint32_t hj = rhh[j] >> (32 - HLL_REG_BITS);
                    const uint32_t rho =
                        (uint32_t)__clz((int)((rhh[j] << HLL_REG_BITS) | (1u << (HLL_REG_BITS - 1)))) + 1;
                    const uint32_t hs = (hj & 3) * 8;
                    uint32_t old = s_hll[hj >> 2];
                    while (rho > ((old >> hs) & 0xFFu)) {
                        const uint32_t nw = (old & ~(0xFFu << hs)) | (rho << hs);
                        const uint32_t prev = atomicCAS(&s_hll[hj >> 2], old, nw);
                        if (prev == old) break;
                        old = prev;
                    }
                }
            }
            wave_sync();
            // lane c < C: bucket c's count -> wave-local start, run reserved in the region of (c, g)
            const unsigned int v = lane < (uint32_t)C ? s_wcnt[wid][lane] : 0u;
            const unsigned int incl = wave_incl_scan(v);
            const unsigned int total = __builtin_amdgcn_readlane(incl, C - 1);
            const unsigned int beg = incl - v;
            // counters restart at the bucket starts: the second round of adds returns positions
            // (the dummy counter at PT_REC: invalid windows land in the dummy slot)
            if (lane <= (uint32_t)C) s_wcnt[wid][lane] = lane < (uint32_t)C ? beg : (unsigned int)PT_REC;
            if (lane < (uint32_t)C) {
                unsigned int at = 0;
                if (v) at = atomicAdd(&s_cur[lane], v);
                unsigned long long b0 = lane * gstride + gcap + at - beg;
                if (at + v > cap) {  // past the capacity: stores go to the spill records, call redone
                    atomicOr(overflow, 1u);
                    b0 = spill - beg;
                }
                s_base[wid][lane] = b0;
            }
            wave_sync();
            unsigned int pos[PT_W];
#pragma unroll
            for (int j = 0; j < PT_W; j++) pos[j] = min(atomicAdd(&s_wcnt[wid][rcb[j]], 1u), (unsigned int)PT_REC);
#pragma unroll
            for (int j = 0; j < PT_W; j++) {
                s_key[wid][pos[j]] = rkey[j];
                s_meta[wid][pos[j]] = rmeta[j];
                s_tag[wid][pos[j]] = (uint8_t)rcb[j];
            }
            wave_sync();
            if (lane <= (uint32_t)C) s_wcnt[wid][lane] = 0;
            unsigned long long ok_[PT_W], ob[PT_W];
            unsigned int om[PT_W];
#pragma unroll
            for (int qq = 0; qq < PT_W; qq++) {
                const unsigned int i = qq * 64 + lane;
                ob[qq] = s_base[wid][s_tag[wid][i] & (C - 1)];
                ok_[qq] = s_key[wid][i];
                om[qq] = s_meta[wid][i];
            }
#pragma unroll
            for (int qq = 0; qq < PT_W; qq++) {
                const unsigned int i = qq * 64 + lane;
                if (i < total) {
                    const unsigned long long idx = ob[qq] + i;
                    keys[idx] = ok_[qq];
                    if (R10)
                        reinterpret_cast<unsigned short *>(metap)[idx] = (unsigned short)om[qq];
                    else
                        reinterpret_cast<unsigned int *>(metap)[idx] = om[qq];
                }
            }
            wave_sync();
        }
    }
    __syncthreads();
    if (threadIdx.x < C) cnt[(uint64_t)threadIdx.x * G + g] = (unsigned int)min((uint64_t)s_cur[threadIdx.x], cap);
    unsigned int *hw = reinterpret_cast<unsigned int *>(hll + g * NREG);
    for (int i = threadIdx.x; i < NREG / 4; i += PT_THREADS) hw[i] = s_hll[i];
}

// HyperLogLog register maxima over the groups' u8 registers (grid: NREG / 256 x TOT_SLICES)
__global__ void __launch_bounds__(256) k_hll_merge(const uint8_t *hll, uint64_t ngroups, unsigned int *hreg) {
    const unsigned int f = blockIdx.x * blockDim.x + threadIdx.x;  // < 2^HLL_REG_BITS
    unsigned int mx = 0;
    for (uint64_t g = blockIdx.y; g < ngroups; g += gridDim.y) mx = max(mx, (unsigned int)hll[g * (1 << HLL_REG_BITS) + f]);
    if (mx) atomicMax(&hreg[f], mx);
}

// ---- refine: region runs of one coarse bucket -> fixed-capacity final buckets ----------------
// Workgroup (c, y) reads the runs of groups [G y / RS, G (y+1) / RS) of coarse bucket c as one
// sequence (run table in LDS), sorts RF_TILE-record tiles by final bucket in LDS and appends each
// final bucket's run at a cursor reserved by one global atomic (fcur[b] counts records stored
// in final bucket b, whose records are [b * fcap, b * fcap + fcur[b]) of `out`, packed 12 B).
constexpr int RF_MAX_RUNS = 2048;
#ifndef RF_TILE
#define RF_TILE 8192  // k_refine2 records per tile (96 KiB of LDS; 4096: 5 % slower)
#endif
// IN10: the input is the partition's R10 records (u64 + u16); the output record then carries
// h = bij_fwd(key) in its key words (k_bucket counts h: Rec12PSource<., true>) and the absolute
// read id (group gsize reads apart) in its meta.
template <bool IN10>
__global__ void __launch_bounds__(BUCKET_THREADS) k_refine2(const unsigned long long *keys, const void *metap,
                                                           const unsigned int *cnt, uint32_t G, uint64_t cap, int bbits,
                                                           unsigned int *out, uint64_t fcap, unsigned long long *fcur,
                                                           unsigned int *overflow, int k, int ibits, uint64_t gsize,
                                                           uint64_t read_base) {
    constexpr int TILE = RF_TILE;
    constexpr int PER = TILE / BUCKET_THREADS;
    __shared__ Rec12 tile[TILE];
    __shared__ uint8_t tj[TILE];
    __shared__ unsigned long long base[REFINE_FANOUT];
    __shared__ unsigned int tcnt[REFINE_FANOUT], tbeg[REFINE_FANOUT], wsum[BUCKET_THREADS / 64];
    __shared__ unsigned int lst[RF_MAX_RUNS + 1];  // run j of the slice = logical [lst[j], lst[j+1])
    const int F = 1 << (bbits - PT_CBITS);
    const uint64_t c = blockIdx.x;
    const uint32_t ga = (uint32_t)((uint64_t)G * blockIdx.y / gridDim.y),
                   gb = (uint32_t)((uint64_t)G * (blockIdx.y + 1) / gridDim.y);
    const uint32_t nr = gb - ga;  // <= RF_MAX_RUNS (host)
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    // exclusive scan of the run lengths (two per thread)
    {
        const uint32_t i0 = 2 * threadIdx.x;
        const unsigned int a = i0 < nr ? cnt[c * G + ga + i0] : 0u, b = i0 + 1 < nr ? cnt[c * G + ga + i0 + 1] : 0u;
        unsigned int incl = a + b;
        for (int o = 1; o < 64; o <<= 1) {
            const unsigned int u = __shfl_up(incl, o);
            if (lane >= o) incl += u;
        }
        if (lane == 63) wsum[wid] = incl;
        __syncthreads();
        unsigned int before = 0;
        for (int q = 0; q < wid; q++) before += wsum[q];
        const unsigned int ex = before + incl - (a + b);
        if (i0 <= nr) lst[i0] = ex;
        if (i0 + 1 <= nr) lst[i0 + 1] = ex + a;
        __syncthreads();
    }
    const uint64_t N = lst[nr];
    constexpr uint64_t C = 1 << PT_CBITS;
    auto phys = [&](uint32_t jrun, uint64_t l) { return ((ga + jrun) * C + c) * cap + (l - lst[jrun]); };
    uint32_t j0 = 0;  // run holding the tile's first record (wave-uniform: every thread tracks it)
    for (uint64_t t0 = 0; t0 < N; t0 += TILE) {
        while (j0 + 1 < nr && lst[j0 + 1] <= t0) j0++;
        const unsigned int n = (unsigned int)min((uint64_t)TILE, N - t0);
        if (threadIdx.x < REFINE_FANOUT) tcnt[threadIdx.x] = 0;
        __syncthreads();
        Rec12 rr[PER];
        unsigned int jj[PER], rk[PER];
        // all loads of the tile first (their waits then overlap), decode after
        unsigned long long lk[PER];
        unsigned int lm[PER], lr[PER];
#pragma unroll
        for (int q = 0; q < PER; q++) {
            const unsigned int i = threadIdx.x + q * BUCKET_THREADS;
            if (i < n) {
                const uint64_t l = t0 + i;
                uint32_t jr = j0;
                while (lst[jr + 1] <= l) jr++;
                const uint64_t p = phys(jr, l);
                lk[q] = keys[p];
                lm[q] = IN10 ? (unsigned int)reinterpret_cast<const unsigned short *>(metap)[p]
                             : reinterpret_cast<const unsigned int *>(metap)[p];
                lr[q] = jr;
            }
        }
#pragma unroll
        for (int q = 0; q < PER; q++) {
            const unsigned int i = threadIdx.x + q * BUCKET_THREADS;
            if (i < n) {
                const unsigned long long kk = lk[q];
                if (IN10) {
                    const int rb1 = 2 * k - PT_CBITS;
                    const uint32_t mbits = ibits + 1;
                    const uint32_t m1 = ((uint32_t)(kk >> rb1) << 16) | lm[q];
                    const uint64_t h = (c << rb1) | (kk & ((1ull << rb1) - 1));
                    rr[q].klo = (unsigned int)h;
                    rr[q].khi = (unsigned int)(h >> 32);
                    rr[q].meta = (uint32_t)((read_base + (uint64_t)(ga + lr[q]) * gsize + (m1 >> mbits)) << mbits) |
                                 (m1 & ((1u << mbits) - 1));
                } else {
                    rr[q].klo = (unsigned int)kk;
                    rr[q].khi = (unsigned int)(kk >> 32);
                    rr[q].meta = lm[q];
                }
            }
        }
#pragma unroll
        for (int q = 0; q < PER; q++) {
            const unsigned int i = threadIdx.x + q * BUCKET_THREADS;
            if (i < n) {
                jj[q] = (IN10 ? (uint32_t)(rkey(rr[q]) >> (2 * k - bbits)) : rec_bucket(rr[q], bbits)) & (F - 1);
                rk[q] = atomicAdd(&tcnt[jj[q]], 1u);
            }
        }
        __syncthreads();
        unsigned long long mybase = 0;
        unsigned int myv = 0;
        if (threadIdx.x < REFINE_FANOUT) {
            const unsigned int v = (int)threadIdx.x < F ? tcnt[threadIdx.x] : 0u;
            unsigned int incl = v;
            for (int o = 1; o < 64; o <<= 1) {
                const unsigned int u = __shfl_up(incl, o);
                if (lane >= o) incl += u;
            }
            tbeg[threadIdx.x] = incl - v;
            if (lane == 63) wsum[wid] = incl;
            myv = v;
            if (v) mybase = atomicAdd(&fcur[c * F + threadIdx.x], (unsigned long long)v);
        }
        __syncthreads();
        if (threadIdx.x >= 64 && threadIdx.x < REFINE_FANOUT) {
            unsigned int add = 0;
            for (int w = 0; w < (int)(threadIdx.x >> 6); w++) add += wsum[w];
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
        if (threadIdx.x < REFINE_FANOUT) {
            if (mybase + myv > fcap) atomicOr(overflow, 1u);  // the records past fcap are dropped
            base[threadIdx.x] = (c * F + threadIdx.x) * fcap + mybase;
            tcnt[threadIdx.x] = mybase < fcap ? (unsigned int)min<unsigned long long>(fcap - mybase, 0xFFFFFFFFull) : 0u;
        }
        __syncthreads();
        for (unsigned int i = threadIdx.x; i < n; i += BUCKET_THREADS) {
            const unsigned int j = tj[i];
            const unsigned int q = i - tbeg[j];
            if (q < tcnt[j]) {
                const uint64_t o = base[j] + q;
                const Rec12 r = tile[i];
                out[3 * o] = r.klo;
                out[3 * o + 1] = r.khi;
                out[3 * o + 2] = r.meta;
            }
        }
        __syncthreads();
    }
}

// k_bucket bounds of the fixed-capacity final buckets: records [b * fcap, b * fcap + fcur[b])
__global__ void __launch_bounds__(256) k_fixed_bounds(const unsigned long long *fcur, uint64_t nb, uint64_t fcap,
                                                      unsigned long long *bbeg, unsigned long long *bend) {
    for (uint64_t b = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; b < nb; b += (uint64_t)gridDim.x * blockDim.x) {
        bbeg[b] = b * fcap;
        bend[b] = b * fcap + min((uint64_t)fcur[b], fcap);
    }
}

}  // namespace ec
