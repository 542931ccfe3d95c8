// assemble.hip -- fused, device-resident restatement of the reference CPU assembler
//   build()        src/referenceassembler/referenceAssembler.py:25-42
//   all_contigs()  src/referenceassembler/referenceAssembler.py:79-111
// on MI355X (gfx950).  The reference walks an insertion-ordered Python dict sequentially;
// here every step is data-parallel and the dict order is recovered from per-string
// first-occurrence events (see DESIGN.md "Parallel formulation"):
//
//   prescan  thread/read : alphabet check, P, HyperLogLog(canonical)       -> table size
//   count    thread/read : rolling 2-bit fwd/rc codes, canonical key, open-addressing
//                          insert (64-bit CAS), count += 1|2, atomicMin first events
//   compact  thread/slot : count > limit -> dense solid arrays (wave ballot + 1 atomic/block)
//   links    thread/node : 8 neighbour probes -> out-degree + unique candidate, then the
//                          get_contig_forward extension rule -> succ / pred (oriented nodes)
//   rank     thread/node : Wyllie pointer jumping (head, rank, prefix-min of first events,
//                          cycle min-id + distance)
//   starts   thread/node : component start = oriented k-mer with the smallest first event
//                          (= first dict entry of its unitig); sort starts -> contig order
//   emit     thread/node : closed-form position of every node in its contig walk
//   gfa      thread/contig: heads/tails lookups -> G
#include "common.h"

#include <rocprim/rocprim.hpp>

#include <algorithm>
#include <cmath>
#include <vector>

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

constexpr int HLL_BITS = 12;
constexpr int HLL_M = 1 << HLL_BITS;
constexpr int MAX_PROBE = 1 << 14;

// sequential byte reader over aligned 32-bit words (an aligned word never crosses a page,
// so reading the word that holds a valid byte is always in-bounds of the allocation)
struct ByteReader {
    uint64_t base;  // absolute address of byte 0
    uint64_t wpos;
    uint32_t word;
    __device__ ByteReader(const uint8_t *b) : base((uint64_t)b), wpos(~0ull), word(0) {}
    __device__ inline uint32_t operator()(uint64_t pos) {
        const uint64_t addr = base + pos;
        const uint64_t a = addr & ~3ull;
        if (a != wpos) {
            wpos = a;
            word = *reinterpret_cast<const uint32_t *>(a);
        }
        return (word >> ((addr & 3) * 8)) & 0xFFu;
    }
};

// Iterate the windows of read r in reference insertion order (build:27-35).  For every
// valid window calls fn(fwd, rc, ef, er): fwd/rc = 2-bit codes of the window and of its
// twin, ef/er = the dict insertion events of the forward string (build:31-32) and of the
// twin string (build:33-35, window j of twin(seg) is the twin of forward window m-1-j).
// Event = (read << 32) | local, local = 2*wb + i (forward) or 2*wb + 2m-1-i (twin).
template <typename Fn>
__device__ inline uint32_t for_each_window(ByteReader &rd, uint64_t s, uint64_t len, int k,
                                           uint64_t r, Fn &&fn) {
    const uint64_t mask = kmask64(k);
    const int sh = 2 * (k - 1);
    uint32_t wb = 0;
    uint64_t p = 0;
    while (p < len) {
        uint64_t q = p;
        while (q < len && base_code(rd(s + q)) < 4) q++;
        if (q - p >= (uint64_t)k) {
            const uint32_t m = (uint32_t)(q - p - k + 1);
            uint64_t fwd = 0, rc = 0;
            for (uint64_t t = p; t < q; t++) {
                const uint64_t b = base_code(rd(s + t));
                fwd = ((fwd << 2) | b) & mask;
                rc = (rc >> 2) | ((3ull - b) << sh);
                if (t - p + 1 >= (uint64_t)k) {
                    const uint32_t i = (uint32_t)(t - p + 1 - k);
                    const uint64_t ef = (r << 32) | (uint64_t)(2 * wb + i);
                    const uint64_t er = (r << 32) | (uint64_t)(2 * wb + 2 * m - 1 - i);
                    fn(fwd, rc, ef, er);
                }
            }
            wb += m;
        }
        p = q + 1;
    }
    return wb;
}

// ---------------------------------------------------------------------------------------
// prescan: alphabet, positions, HyperLogLog registers (one LDS copy per block)
__global__ void __launch_bounds__(256) k_prescan(const uint8_t *buf, const uint64_t *off, uint64_t nreads,
                                                 int k, uint8_t *hll_blocks, unsigned long long *npos,
                                                 unsigned long long *bad) {
    __shared__ uint32_t reg[HLL_M];
    for (int i = threadIdx.x; i < HLL_M; i += blockDim.x) reg[i] = 0;
    __syncthreads();
    unsigned long long mypos = 0;
    for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < nreads;
         r += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t s = off[r], len = off[r + 1] - s;
        ByteReader rd(buf);
        for (uint64_t t = 0; t < len; t++) {
            if (base_code(rd(s + t)) == 5) {
                atomicMin(bad, (unsigned long long)(s + t));
                break;
            }
        }
        mypos += for_each_window(rd, s, len, k, r, [&](uint64_t fwd, uint64_t rc, uint64_t, uint64_t) {
            const uint64_t c = fwd < rc ? fwd : rc;
            const uint64_t h = mix64(c);
            const uint32_t j = (uint32_t)(h >> (64 - HLL_BITS));
            const uint64_t w = (h << HLL_BITS) | (1ull << (HLL_BITS - 1));
            const uint32_t rho = (uint32_t)__clzll((long long)w) + 1;
            atomicMax(&reg[j], rho);
        });
    }
    // block reduce positions
    for (int o = 32; o > 0; o >>= 1) mypos += __shfl_down(mypos, o);
    if ((threadIdx.x & 63) == 0 && mypos) atomicAdd(npos, mypos);
    __syncthreads();
    for (int i = threadIdx.x; i < HLL_M; i += blockDim.x) hll_blocks[(uint64_t)blockIdx.x * HLL_M + i] = (uint8_t)reg[i];
}

__global__ void __launch_bounds__(1024) k_hll_final(const uint8_t *hll_blocks, int nblocks, double *est) {
    __shared__ double red[1024];
    __shared__ int zeros[1024];
    double sum = 0;
    int z = 0;
    for (int j = threadIdx.x; j < HLL_M; j += blockDim.x) {
        uint32_t m = 0;
        for (int b = 0; b < nblocks; b++) m = max(m, (uint32_t)hll_blocks[(uint64_t)b * HLL_M + j]);
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
        const double m = HLL_M;
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
                                               Slot *table, uint64_t capmask, unsigned int *overflow) {
    for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < nreads;
         r += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t s = off[r], len = off[r + 1] - s;
        ByteReader rd(buf);
        for_each_window(rd, s, len, k, r, [&](uint64_t fwd, uint64_t rc, uint64_t ef, uint64_t er) {
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

// compact: solid (count > limit, build:37-39) slots -> dense arrays
__global__ void __launch_bounds__(256) k_compact(Slot *table, uint64_t cap, long long limit,
                                                 unsigned long long *dkey, unsigned int *dcnt,
                                                 unsigned long long *dfc, unsigned long long *dft,
                                                 unsigned int *nsolid, unsigned long long *ndistinct) {
    __shared__ unsigned int wave_cnt[4];
    __shared__ unsigned int base;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (uint64_t i0 = blockIdx.x * (uint64_t)blockDim.x; i0 < cap; i0 += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t i = i0 + threadIdx.x;
        Slot sl;
        bool present = false, solid = false;
        if (i < cap) {
            sl = table[i];
            present = sl.key != EMPTY_KEY;
            solid = present && (long long)sl.count > limit;
        }
        const unsigned long long m = __ballot(solid);
        const unsigned long long mp = __ballot(present);
        const unsigned int before = __popcll(m & ((1ull << lane) - 1));
        if (lane == 0) {
            wave_cnt[wid] = __popcll(m);
            if (mp) atomicAdd(ndistinct, (unsigned long long)__popcll(mp));
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned int tot = 0;
            for (int w = 0; w < 4; w++) {
                unsigned int c = wave_cnt[w];
                wave_cnt[w] = tot;
                tot += c;
            }
            base = tot ? atomicAdd(nsolid, tot) : 0;
        }
        __syncthreads();
        if (solid) {
            const unsigned int u = base + wave_cnt[wid] + before;
            dkey[u] = sl.key;
            dcnt[u] = sl.count;
            dfc[u] = sl.fC;
            dft[u] = sl.fT;
            table[i].idx = u;
        }
        __syncthreads();
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

// oriented node id: 2u + o (o = 1: twin of the canonical string); palindromes use o = 0 only
__device__ inline uint64_t node_code(const unsigned long long *dkey, unsigned int x, int k) {
    const uint64_t c = dkey[x >> 1];
    return (x & 1) ? twin64(c, k) : c;
}
__device__ inline unsigned int twin_node(const uint8_t *upal, unsigned int x) {
    return upal[x >> 1] ? x : (x ^ 1u);
}

// links phase 1: out-degree (number of fw(x) in d, get_contig_forward:63) + the unique candidate
__global__ void __launch_bounds__(256) k_neighbors(const Slot *table, uint64_t capmask, const unsigned long long *dkey,
                                                   unsigned int U, int k, uint8_t *upal, uint8_t *outdeg,
                                                   unsigned int *cand, unsigned int *npal) {
    const uint64_t mask = kmask64(k);
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < 2ull * U; t += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned int x = (unsigned int)t;
        const uint64_t c = dkey[x >> 1];
        const uint64_t tc = twin64(c, k);
        const bool pal = tc == c;
        if (x & 1) {
            if (pal) {  // the palindrome has a single dict entry: node 2u+1 does not exist
                outdeg[x] = 0;
                cand[x] = NONE32;
                continue;
            }
        } else {
            upal[x >> 1] = pal ? 1 : 0;
            if (pal) atomicAdd(npal, 1u);
        }
        const uint64_t xs = (x & 1) ? tc : c;
        unsigned int n = 0, cd = NONE32;
        for (int b = 0; b < 4; b++) {
            const uint64_t y = ((xs << 2) | (uint64_t)b) & mask;
            const uint64_t ty = twin64(y, k);
            const uint64_t cy = y < ty ? y : ty;
            const unsigned int u = lookup(table, capmask, cy);
            if (u != NONE32) {
                if (n == 0) cd = 2 * u + (y != cy ? 1u : 0u);
                n++;
            }
        }
        outdeg[x] = (uint8_t)n;
        cand[x] = n == 1 ? cd : NONE32;
    }
}

// links phase 2: x -> y iff |fw(x) in d| == 1, |bw(y) in d| == 1 and y != twin(x)
// (get_contig_forward:63-73; the cand == km / twin(km) stop is applied by the walk emulation)
// |bw(y) in d| == |fw(twin y) in d| == outdeg[twin y].
__global__ void __launch_bounds__(256) k_succ(const uint8_t *upal, const uint8_t *outdeg, const unsigned int *cand,
                                              unsigned int N, unsigned int *succ) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < N; t += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned int x = (unsigned int)t;
        unsigned int s = NONE32;
        const unsigned int y = cand[x];
        if (y != NONE32 && !((x & 1) && upal[x >> 1])) {
            const unsigned int ty = twin_node(upal, y);
            if (outdeg[ty] == 1 && y != twin_node(upal, x)) s = y;
        }
        succ[x] = s;
    }
}

__device__ inline unsigned long long first_event(const unsigned long long *dfc, const unsigned long long *dft,
                                                 unsigned int x) {
    return (x & 1) ? dft[x >> 1] : dfc[x >> 1];
}

// pred(x) = twin(succ(twin(x))): the links are closed under twin-reversal
__global__ void __launch_bounds__(256) k_pred(const uint8_t *upal, const unsigned int *succ, unsigned int N,
                                              unsigned int *pred) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < N; t += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned int x = (unsigned int)t;
        unsigned int p = NONE32;
        if (!((x & 1) && upal[x >> 1])) {
            const unsigned int sx = succ[twin_node(upal, x)];
            if (sx != NONE32) p = twin_node(upal, sx);
        }
        pred[x] = p;
    }
}

// ---- list ranking by a sparse ruling set ------------------------------------------------
// Rulers: every path head plus every node whose hash hits the sampling mask.  Each ruler
// walks its segment (up to the next ruler) serially, stamping (ruler, offset) on every node;
// the much shorter ruler list is then ranked by weighted Wyllie pointer jumping.  Cycles
// that drew no ruler are caught by later iterations with a denser sampling mask (the last
// one makes every still-unvisited node a ruler).
__device__ inline bool ruler_hash(unsigned int x, unsigned int smask) {
    return (mix64(0x9E3779B97F4A7C15ull ^ x) & smask) == 0;
}

__global__ void __launch_bounds__(256) k_rulers(const uint8_t *upal, const unsigned int *pred, unsigned int N,
                                                unsigned int smask, int first, unsigned int *rid, unsigned int *roff,
                                                unsigned int *rlist, unsigned int *nr) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < N; t += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned int x = (unsigned int)t;
        if ((x & 1) && upal[x >> 1]) continue;
        if (rid[x] != NONE32) continue;
        if ((first && pred[x] == NONE32) || ruler_hash(x, smask)) {
            const unsigned int i = atomicAdd(nr, 1u);
            rlist[i] = x;
            rid[x] = i;
            roff[x] = 0;
        }
    }
}

// ruler jump state (32 B): window = rulers i, P(i), .., P^{c-1}(i)
struct alignas(32) RJump {
    unsigned int a;    // P^c(i) or NONE
    unsigned int s;    // nodes in the segments of P(i)..P^{c-1}(i)  (= rank of i's node on a path)
    unsigned int h;    // last ruler of the window (the head ruler once a == NONE)
    unsigned int cm;   // min ruler node id in the window
    unsigned int cd;   // nodes from cm forward to i's node
    unsigned int len;  // nodes in i's own segment
    unsigned long long fm;  // min first event over the window's segments (incl. i's)
};
static_assert(sizeof(RJump) == 32, "rjump layout");

__global__ void __launch_bounds__(256) k_walk(const unsigned int *succ, const unsigned long long *dfc,
                                              const unsigned long long *dft, const unsigned int *rlist,
                                              unsigned int r0, const unsigned int *nr, unsigned int smask,
                                              unsigned int *rid, unsigned int *roff, unsigned int *nextR, RJump *rs,
                                              unsigned long long *nvisited) {
    const unsigned int r1 = *nr;
    unsigned long long seen = 0;
    for (uint64_t t = r0 + blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < r1; t += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned int i = (unsigned int)t;
        unsigned int v = rlist[i];
        unsigned long long fm = first_event(dfc, dft, v);
        unsigned int j = 0, nx = NONE32;
        for (;;) {
            const unsigned int w = succ[v];
            if (w == NONE32) break;
            if (ruler_hash(w, smask) && rid[w] != NONE32) {  // the next ruler
                nx = rid[w];
                break;
            }
            v = w;
            j++;
            rid[v] = i;
            roff[v] = j;
            const unsigned long long f = first_event(dfc, dft, v);
            fm = f < fm ? f : fm;
        }
        nextR[i] = nx;
        RJump r;
        r.a = NONE32;  // set from prevR by k_rjump_init
        r.s = 0;
        r.h = i;
        r.cm = rlist[i];
        r.cd = 0;
        r.len = j + 1;
        r.fm = fm;
        rs[i] = r;
        seen += j + 1;
    }
    for (int o = 32; o > 0; o >>= 1) seen += __shfl_down(seen, o);
    if ((threadIdx.x & 63) == 0 && seen) atomicAdd(nvisited, seen);
}

__global__ void __launch_bounds__(256) k_rjump_init(const unsigned int *nextR, unsigned int nr, RJump *rs) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < nr; t += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned int n = nextR[t];
        if (n != NONE32) rs[n].a = (unsigned int)t;  // prevR[next] = me (unique predecessor)
    }
}

// one weighted Wyllie round on the ruler list
__global__ void __launch_bounds__(256) k_rjump(const RJump *src, RJump *dst, unsigned int nr, unsigned int N,
                                               const unsigned int *active_in, unsigned int *active_out,
                                               unsigned int *final_sel, unsigned int sel) {
    if (active_in && *active_in == 0) return;
    unsigned int act = 0;
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < nr; t += (uint64_t)gridDim.x * blockDim.x) {
        RJump j = src[t];
        if (j.a != NONE32 && j.s < N) {
            const RJump y = src[j.a];
            const unsigned int back = j.s + y.len;  // nodes from ruler a's node forward to i's node
            if (y.cm < j.cm) {
                j.cm = y.cm;
                j.cd = back + y.cd;
            }
            j.s = back + y.s;
            j.a = y.a;
            j.h = y.h;
            j.fm = y.fm < j.fm ? y.fm : j.fm;
            act += (j.a != NONE32 && j.s < N);
        }
        dst[t] = j;
    }
    for (int o = 32; o > 0; o >>= 1) act += __shfl_down(act, o);
    if ((threadIdx.x & 63) == 0 && act) atomicAdd(active_out, act);
    if (blockIdx.x == 0 && threadIdx.x == 0) *final_sel = sel;
}

// per-node path descriptor: PK = path key (head node for paths, min ruler node for cycles)
// with bit 31 = on a cycle; RK = rank (from the head / from the cycle key).  Path records
// at the key node: PL = path / cycle length, PM = min first event over it.
constexpr unsigned int CYC = 0x80000000u;

__global__ void __launch_bounds__(256) k_finalize(const uint8_t *upal, const unsigned int *succ, const unsigned int *rid,
                                                  const unsigned int *roff, const unsigned int *rlist, const RJump *rs,
                                                  unsigned int N, unsigned int *PK, unsigned int *RK, unsigned int *PL,
                                                  unsigned long long *PM) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < N; t += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned int x = (unsigned int)t;
        if ((x & 1) && upal[x >> 1]) continue;
        const unsigned int i = rid[x], j = roff[x];
        const RJump r = rs[i];
        if (r.a == NONE32) {  // path
            const unsigned int pk = rlist[r.h], rk = r.s + j;
            PK[x] = pk;
            RK[x] = rk;
            if (succ[x] == NONE32) {  // tail: its ruler's window spans the whole path
                PL[pk] = rk + 1;
                PM[pk] = r.fm;
            }
        } else {  // cycle
            PK[x] = r.cm | CYC;
            RK[x] = r.cd + j;
        }
    }
}

// cycle length / min: the ruler whose successor ruler is the key ruler closes the ring
__global__ void __launch_bounds__(256) k_cycle_len(const unsigned int *nextR, const unsigned int *rlist, const RJump *rs,
                                                   unsigned int nr, unsigned int *PL, unsigned long long *PM) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < nr; t += (uint64_t)gridDim.x * blockDim.x) {
        const RJump r = rs[t];
        if (r.a == NONE32) continue;
        const unsigned int n = nextR[t];
        if (n != NONE32 && rlist[n] == r.cm) {
            PL[r.cm] = r.cd + r.len;
            PM[r.cm] = r.fm;
        }
    }
}

__device__ inline unsigned long long path_min(const unsigned int *PK, const unsigned long long *PM, unsigned int x) {
    return PM[PK[x] & ~CYC];
}

// start of each component (all_contigs:82-84): the oriented k-mer with the smallest first
// event over the path and its twin path (= the first dict entry not yet `done`).
__global__ void __launch_bounds__(256) k_starts(const uint8_t *upal, const unsigned long long *dfc,
                                                const unsigned long long *dft, const unsigned int *PK,
                                                const unsigned long long *PM, unsigned int N,
                                                unsigned long long *skeys, unsigned int *svals, unsigned int *nstarts) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < N; t += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned int x = (unsigned int)t;
        if ((x & 1) && upal[x >> 1]) continue;
        const unsigned long long f = first_event(dfc, dft, x);
        const unsigned long long a = path_min(PK, PM, x);
        const unsigned long long b = path_min(PK, PM, twin_node(upal, x));
        if (f == (a < b ? a : b)) {
            const unsigned int i = atomicAdd(nstarts, 1u);
            skeys[i] = f;
            svals[i] = x;
        }
    }
}

// geometry of the walk from start s (get_contig:47-56 + get_contig_forward:59-77):
//   kind 0 path, twin path disjoint   : contig = the path holding s, head..tail
//   kind 1 path equal to its twin     : p_0..p_n, s = p_j : p_0..p_{n-j-1} | p_{n-j+1}..p_n | all
//   kind 2 cycle, twin cycle disjoint : s, succ(s), ... (n nodes)
//   kind 3 cycle equal to its twin    : m = dist(s -> twin s): m == 0 -> all n from s,
//                                       else p_{m+1}..p_{n-1}, p_0..p_{m-1} (n-1 nodes)
struct Walk {
    unsigned int kind, n, j, m, lo, len;
};

__device__ inline Walk walk_of(const uint8_t *upal, const unsigned int *PK, const unsigned int *RK,
                               const unsigned int *PL, unsigned int s) {
    Walk w;
    const unsigned int pk = PK[s], rk = RK[s];
    const unsigned int ts = twin_node(upal, s);
    const unsigned int pk2 = PK[ts], rk2 = RK[ts];
    const bool self = pk2 == pk;
    const unsigned int plen = PL[pk & ~CYC];
    w.j = rk;
    w.m = 0;
    w.lo = 0;
    if (!(pk & CYC)) {
        if (!self) {
            w.kind = 0;
            w.n = plen;
            w.len = plen;
        } else {
            w.kind = 1;
            const unsigned int n = plen - 1, j = rk;
            w.n = n;
            if (2 * j < n) {
                w.lo = 0;
                w.len = n - j;
            } else if (2 * j > n) {
                w.lo = n - j + 1;
                w.len = j;
            } else {
                w.lo = 0;
                w.len = n + 1;
            }
        }
    } else {
        const unsigned int n = plen;
        w.n = n;
        if (!self) {
            w.kind = 2;
            w.len = n;
        } else {
            w.kind = 3;
            w.m = (rk2 + n - rk) % n;
            w.len = w.m == 0 ? n : n - 1;
        }
    }
    return w;
}

__global__ void __launch_bounds__(256) k_contig_len(const uint8_t *upal, const unsigned int *PK, const unsigned int *RK,
                                                    const unsigned int *PL, const unsigned int *sorted_nodes,
                                                    unsigned int nc, int k, unsigned int *cidxOf,
                                                    unsigned long long *clen) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nc; i += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned int s = sorted_nodes[i];
        cidxOf[PK[s] & ~CYC] = (unsigned int)i;
        const Walk w = walk_of(upal, PK, RK, PL, s);
        clen[i] = (unsigned long long)(k - 1) + w.len;
    }
}

// emit: every node finds its contig through its path key, computes its walk position and
// writes its chars (contig_to_string:44-45: first node k chars, later nodes their last base).
__global__ void __launch_bounds__(256) k_emit(const uint8_t *upal, const unsigned int *PK, const unsigned int *RK,
                                              const unsigned int *PL, const unsigned long long *dkey,
                                              const unsigned int *cidxOf, const unsigned int *sorted_nodes,
                                              const unsigned long long *coff, unsigned int N, int k, char *chars,
                                              unsigned int *cfirst, unsigned int *clast, unsigned int *headOf,
                                              unsigned int *tailOf) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < N; t += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned int x = (unsigned int)t;
        if ((x & 1) && upal[x >> 1]) continue;
        const unsigned int pk = PK[x], rk = RK[x];
        const unsigned int ci = cidxOf[pk & ~CYC];
        if (ci == NONE32) continue;  // the twin path of a disjoint pair carries the contig
        const unsigned int s = sorted_nodes[ci];
        const Walk w = walk_of(upal, PK, RK, PL, s);
        long long pos = -1;
        if (w.kind == 0) {
            pos = rk;
        } else if (w.kind == 1) {
            if (rk >= w.lo && rk < w.lo + w.len) pos = rk - w.lo;
        } else {
            const unsigned int i = (rk + w.n - w.j) % w.n;  // steps from s
            if (w.kind == 2 || w.m == 0) {
                pos = i;
            } else if (i > w.m) {
                pos = i - w.m - 1;
            } else if (i < w.m) {
                pos = w.n - 1 - w.m + i;
            }
        }
        if (pos < 0) continue;
        const uint64_t code = node_code(dkey, x, k);
        char *dst = chars + coff[ci];
        if (pos == 0) {
            uint64_t c = code;
            for (int i = k - 1; i >= 0; i--) {
                dst[i] = "ACGT"[c & 3];
                c >>= 2;
            }
            cfirst[ci] = x;
            headOf[x] = ci;
        } else {
            dst[k - 1 + pos] = "ACGT"[code & 3];
        }
        if ((unsigned long long)pos == (unsigned long long)w.len - 1) {
            clast[ci] = x;
            tailOf[twin_node(upal, x)] = ci;
        }
    }
}

// GFA links (all_contigs:90-109): for y in fw(last kmer): heads[y] then tails[y];
// for z in fw(twin(first kmer)): heads[z] then tails[z].  Up to 8 per side.
__global__ void __launch_bounds__(256) k_gfa(const Slot *table, uint64_t capmask, const unsigned long long *dkey,
                                             const uint8_t *upal, const unsigned int *cfirst, const unsigned int *clast,
                                             const unsigned int *headOf, const unsigned int *tailOf, unsigned int nc,
                                             int k, long long *lk, unsigned int *lcnt) {
    const uint64_t mask = kmask64(k);
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nc; i += (uint64_t)gridDim.x * blockDim.x) {
        for (int side = 0; side < 2; side++) {
            const unsigned int src = side == 0 ? clast[i] : twin_node(upal, cfirst[i]);
            const uint64_t xs = node_code(dkey, src, k);
            unsigned int n = 0;
            long long *o = lk + (i * 2 + side) * 8;
            for (int b = 0; b < 4; b++) {
                const uint64_t y = ((xs << 2) | (uint64_t)b) & mask;
                const uint64_t ty = twin64(y, k);
                const uint64_t cy = y < ty ? y : ty;
                const unsigned int u = lookup(table, capmask, cy);
                if (u == NONE32) continue;
                const unsigned int oy = (y != cy) ? 2 * u + 1 : 2 * u;
                const unsigned int hh = headOf[oy], tt = tailOf[oy];
                if (hh != NONE32) o[n++] = 2ll * hh;
                if (tt != NONE32) o[n++] = 2ll * tt + 1;
            }
            lcnt[i * 2 + side] = n;
        }
    }
}

// ordered dict of build(): every valid oriented node with its first event (sort key)
__global__ void __launch_bounds__(256) k_dict_items(const uint8_t *upal, const unsigned long long *dfc,
                                                    const unsigned long long *dft, unsigned int N,
                                                    unsigned long long *keys, unsigned int *vals, unsigned int *n) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < N; t += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned int x = (unsigned int)t;
        if ((x & 1) && upal[x >> 1]) continue;
        const unsigned int i = atomicAdd(n, 1u);
        keys[i] = first_event(dfc, dft, x);
        vals[i] = x;
    }
}

__global__ void __launch_bounds__(256) k_dict_render(const unsigned int *nodes, unsigned int n,
                                                     const unsigned long long *dkey, const unsigned int *dcnt, int k,
                                                     char *out, unsigned int *counts) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned int x = nodes[i];
        uint64_t c = node_code(dkey, x, k);
        for (int p = k - 1; p >= 0; p--) {
            out[i * k + p] = "ACGT"[c & 3];
            c >>= 2;
        }
        counts[i] = dcnt[x >> 1];
    }
}

// ---------------------------------------------------------------------------------------
// host side
struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    int ensure(size_t bytes) {
        if (bytes <= cap) return EC_OK;
        if (p) hipFree(p);
        p = nullptr;
        cap = 0;
        size_t want = std::max<size_t>(bytes, 256);
        if (hipMalloc(&p, want) != hipSuccess) {
            set_error("hipMalloc(%zu) failed", want);
            return EC_ERR_NOMEM;
        }
        cap = want;
        return EC_OK;
    }
    template <typename T>
    T *as() const { return reinterpret_cast<T *>(p); }
    void release() {
        if (p) hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

}  // namespace ec

using namespace ec;

struct ec_session {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    // scratch
    DevBuf h_reads, h_offsets;  // H2D staging for ec_assemble_host
    DevBuf hll, scal, table, dkey, dcnt, dfc, dft, upal, outdeg, cand, succ, pred, st0, st1;
    DevBuf rid, roff, rlist, nextR, PK, RK, PL, PM;
    DevBuf startOf, skeys, svals, skeys2, svals2, cidxOf, clen, coff, chars, cfirst, clast, headOf, tailOf;
    DevBuf lk, lcnt, tmp, dchars, dcounts;
    // results (host)
    bool have = false;
    int k = 0;
    ec_stats stats{};
    std::vector<char> h_chars;
    std::vector<uint64_t> h_coff;
    std::vector<uint64_t> h_loff;
    std::vector<int64_t> h_links;
    bool want_dict = false;
    hipEvent_t ev[2 * EC_NSTAGES + 2] = {};
    bool events = false;
};

namespace {

struct Scalars {  // device scalars block
    unsigned long long npos;
    unsigned long long bad;
    unsigned long long ndistinct;
    double est;
    unsigned int overflow;
    unsigned int nsolid;
    unsigned int nstarts;
    unsigned int final_sel;
    unsigned int ndict;
    unsigned int nr;
    unsigned int npal;
    unsigned int pad;
    unsigned long long nvisited;
    unsigned int active[64];
};

int scan_u64(ec_session *s, const unsigned long long *in, unsigned long long *out, size_t n) {
    size_t bytes = 0;
    EC_HIP(rocprim::exclusive_scan(nullptr, bytes, in, out, 0ull, n, rocprim::plus<unsigned long long>(), s->stream));
    EC_CHECK(s->tmp.ensure(bytes));
    EC_HIP(rocprim::exclusive_scan(s->tmp.p, bytes, in, out, 0ull, n, rocprim::plus<unsigned long long>(), s->stream));
    return EC_OK;
}

int sort_pairs(ec_session *s, unsigned long long *kin, unsigned long long *kout, unsigned int *vin, unsigned int *vout,
               size_t n) {
    size_t bytes = 0;
    EC_HIP(rocprim::radix_sort_pairs(nullptr, bytes, kin, kout, vin, vout, n, 0, 64, s->stream));
    EC_CHECK(s->tmp.ensure(bytes));
    EC_HIP(rocprim::radix_sort_pairs(s->tmp.p, bytes, kin, kout, vin, vout, n, 0, 64, s->stream));
    return EC_OK;
}

inline void mark(ec_session *s, int idx) {
    if (s->events) hipEventRecord(s->ev[idx], s->stream);
}

int assemble(ec_session *s, const uint8_t *d_reads, const uint64_t *d_off, uint64_t nreads, int k, int limit,
             unsigned flags) {
    s->have = false;
    if (k < 1 || k > EC_MAX_K) {
        set_error("k=%d outside [1,%d] (fused path uses 64-bit keys)", k, EC_MAX_K);
        return EC_ERR_ARG;
    }
    if (nreads >= (1ull << 32)) {
        set_error("nreads=%llu >= 2^32", (unsigned long long)nreads);
        return EC_ERR_ARG;
    }
    EC_HIP(hipSetDevice(s->device));
    memset(&s->stats, 0, sizeof(s->stats));
    s->stats.n_reads = nreads;
    s->k = k;
    s->want_dict = (flags & EC_FLAG_WANT_DICT) != 0;
    const bool timing = (flags & EC_FLAG_TIMING) != 0;
    if (timing && !s->events) {
        for (auto &e : s->ev) EC_HIP(hipEventCreate(&e));
        s->events = true;
    }
    bool saved_events = s->events;
    if (!timing) s->events = false;
    hipStream_t st = s->stream;
    const unsigned B = 256;

    EC_CHECK(s->scal.ensure(sizeof(Scalars)));
    Scalars *dsc = s->scal.as<Scalars>();
    EC_HIP(hipMemsetAsync(dsc, 0, sizeof(Scalars), st));
    EC_HIP(hipMemsetAsync(&dsc->bad, 0xFF, sizeof(unsigned long long), st));
    Scalars hsc;

    // ---- prescan ------------------------------------------------------------------------
    mark(s, 2 * EC_STAGE_PRESCAN);
    const unsigned pre_blocks = grid_for(nreads ? nreads : 1, B, 1024);
    EC_CHECK(s->hll.ensure((size_t)pre_blocks * HLL_M));
    if (nreads) {
        k_prescan<<<pre_blocks, B, 0, st>>>(d_reads, d_off, nreads, k, s->hll.as<uint8_t>(), &dsc->npos, &dsc->bad);
        k_hll_final<<<1, 1024, 0, st>>>(s->hll.as<uint8_t>(), pre_blocks, &dsc->est);
    }
    mark(s, 2 * EC_STAGE_PRESCAN + 1);
    EC_HIP(hipMemcpyAsync(&hsc, dsc, sizeof(Scalars), hipMemcpyDeviceToHost, st));
    EC_HIP(hipStreamSynchronize(st));
    if (hsc.bad != ~0ull) {
        uint8_t byte = 0;
        hipMemcpy(&byte, d_reads + hsc.bad, 1, hipMemcpyDeviceToHost);
        set_error("byte %llu (0x%02x) outside {A,C,G,T,N}", (unsigned long long)hsc.bad, byte);
        s->events = saved_events;
        return EC_ERR_ALPHABET;
    }
    s->stats.n_positions = nreads ? hsc.npos : 0;
    s->stats.n_distinct_est = nreads ? (uint64_t)llround(hsc.est) : 0;

    // ---- count (with capacity retries) ----------------------------------------------------
    uint64_t want = (uint64_t)(std::max<double>(nreads ? hsc.est : 0, 1.0) * 2.2) + 1024;
    want = std::min<uint64_t>(want, 2 * s->stats.n_positions + 1024);
    uint64_t cap = 1024;
    while (cap < want) cap <<= 1;
    for (int attempt = 0;; attempt++) {
        EC_CHECK(s->table.ensure(cap * sizeof(Slot)));
        mark(s, 2 * EC_STAGE_COUNT);
        k_table_clear<<<grid_for(cap, B, 8192), B, 0, st>>>(s->table.as<Slot>(), cap);
        EC_HIP(hipMemsetAsync(&dsc->overflow, 0, 4, st));
        if (timing) hipEventRecord(s->ev[2 * EC_NSTAGES], st);
        if (nreads)
            k_count<<<grid_for(nreads, B), B, 0, st>>>(d_reads, d_off, nreads, k, s->table.as<Slot>(), cap - 1,
                                                      &dsc->overflow);
        if (timing) hipEventRecord(s->ev[2 * EC_NSTAGES + 1], st);
        mark(s, 2 * EC_STAGE_COUNT + 1);
        EC_HIP(hipMemcpyAsync(&hsc.overflow, &dsc->overflow, 4, hipMemcpyDeviceToHost, st));
        EC_HIP(hipStreamSynchronize(st));
        if (!hsc.overflow) break;
        if (attempt >= 4) {
            set_error("hash table overflow at capacity %llu", (unsigned long long)cap);
            s->events = saved_events;
            return EC_ERR_CAPACITY;
        }
        cap <<= 2;
        s->stats.table_retries++;
    }
    s->stats.table_capacity = cap;

    // ---- compact --------------------------------------------------------------------------
    mark(s, 2 * EC_STAGE_COMPACT);
    // dense arrays sized by the distinct estimate bound: at most cap/1 entries
    // (allocate lazily after knowing U is cheaper but needs a sync; size by cap)
    const uint64_t umax = cap;
    EC_CHECK(s->dkey.ensure(umax * 8));
    EC_CHECK(s->dcnt.ensure(umax * 4));
    EC_CHECK(s->dfc.ensure(umax * 8));
    EC_CHECK(s->dft.ensure(umax * 8));
    k_compact<<<grid_for(cap, B, 8192), B, 0, st>>>(s->table.as<Slot>(), cap, (long long)limit,
                                                   s->dkey.as<unsigned long long>(), s->dcnt.as<unsigned int>(),
                                                   s->dfc.as<unsigned long long>(), s->dft.as<unsigned long long>(),
                                                   &dsc->nsolid, &dsc->ndistinct);
    mark(s, 2 * EC_STAGE_COMPACT + 1);
    EC_HIP(hipMemcpyAsync(&hsc, dsc, sizeof(Scalars), hipMemcpyDeviceToHost, st));
    EC_HIP(hipStreamSynchronize(st));
    const unsigned int U = hsc.nsolid;
    s->stats.n_distinct = hsc.ndistinct;
    s->stats.n_solid = U;
    if (2ull * U >= 0xFFFFFFF0ull) {
        set_error("too many solid k-mers (%u) for 32-bit node ids", U);
        s->events = saved_events;
        return EC_ERR_CAPACITY;
    }
    const unsigned int N = 2 * U;
    const size_t Nn = std::max<size_t>(N, 1);

    // ---- links ----------------------------------------------------------------------------
    mark(s, 2 * EC_STAGE_LINKS);
    EC_CHECK(s->upal.ensure(std::max<size_t>(U, 1)));
    EC_CHECK(s->outdeg.ensure(Nn));
    EC_CHECK(s->cand.ensure(Nn * 4));
    EC_CHECK(s->succ.ensure(Nn * 4));
    EC_CHECK(s->pred.ensure(Nn * 4));
    if (U) {
        k_neighbors<<<grid_for(N, B), B, 0, st>>>(s->table.as<Slot>(), cap - 1, s->dkey.as<unsigned long long>(), U, k,
                                                 s->upal.as<uint8_t>(), s->outdeg.as<uint8_t>(),
                                                 s->cand.as<unsigned int>(), &dsc->npal);
        k_succ<<<grid_for(N, B), B, 0, st>>>(s->upal.as<uint8_t>(), s->outdeg.as<uint8_t>(), s->cand.as<unsigned int>(),
                                            N, s->succ.as<unsigned int>());
        k_pred<<<grid_for(N, B), B, 0, st>>>(s->upal.as<uint8_t>(), s->succ.as<unsigned int>(), N,
                                            s->pred.as<unsigned int>());
    }
    mark(s, 2 * EC_STAGE_LINKS + 1);

    // ---- rank (sparse ruling set + weighted Wyllie on the rulers) -------------------------
    mark(s, 2 * EC_STAGE_RANK);
    EC_CHECK(s->rid.ensure(Nn * 4));
    EC_CHECK(s->roff.ensure(Nn * 4));
    EC_CHECK(s->rlist.ensure(Nn * 4));
    EC_CHECK(s->nextR.ensure(Nn * 4));
    EC_CHECK(s->st0.ensure(Nn * sizeof(RJump)));
    EC_CHECK(s->st1.ensure(Nn * sizeof(RJump)));
    EC_CHECK(s->PK.ensure(Nn * 4));
    EC_CHECK(s->RK.ensure(Nn * 4));
    EC_CHECK(s->PL.ensure(Nn * 4));
    EC_CHECK(s->PM.ensure(Nn * 8));
    unsigned int nr = 0;
    RJump *fin = s->st0.as<RJump>();
    s->stats.rank_rounds = 0;
    if (U) {
        EC_HIP(hipMemsetAsync(s->rid.p, 0xFF, Nn * 4, st));
        const unsigned int masks[4] = {31u, 7u, 1u, 0u};
        unsigned int r0 = 0;
        for (int it = 0; it < 4; it++) {
            k_rulers<<<grid_for(N, B), B, 0, st>>>(s->upal.as<uint8_t>(), s->pred.as<unsigned int>(), N, masks[it],
                                                  it == 0, s->rid.as<unsigned int>(), s->roff.as<unsigned int>(),
                                                  s->rlist.as<unsigned int>(), &dsc->nr);
            k_walk<<<2048, B, 0, st>>>(s->succ.as<unsigned int>(), s->dfc.as<unsigned long long>(),
                                      s->dft.as<unsigned long long>(), s->rlist.as<unsigned int>(), r0, &dsc->nr,
                                      masks[it], s->rid.as<unsigned int>(), s->roff.as<unsigned int>(),
                                      s->nextR.as<unsigned int>(), s->st0.as<RJump>(), &dsc->nvisited);
            EC_HIP(hipMemcpyAsync(&hsc, dsc, sizeof(Scalars), hipMemcpyDeviceToHost, st));
            EC_HIP(hipStreamSynchronize(st));
            r0 = hsc.nr;
            if (hsc.nvisited + hsc.npal >= N) break;
        }
        nr = hsc.nr;
        if (hsc.nvisited + hsc.npal != N) {
            set_error("ruling set covered %llu of %u nodes", (unsigned long long)(hsc.nvisited + hsc.npal), N);
            s->events = saved_events;
            return EC_ERR_STATE;
        }
        k_rjump_init<<<grid_for(nr, B), B, 0, st>>>(s->nextR.as<unsigned int>(), nr, s->st0.as<RJump>());
        int rounds = 1;
        while ((1ull << (rounds - 1)) < (unsigned long long)nr) rounds++;
        rounds = std::min(rounds + 1, 63);
        RJump *bufs[2] = {s->st0.as<RJump>(), s->st1.as<RJump>()};
        for (int r = 0; r < rounds; r++)
            k_rjump<<<grid_for(nr, B), B, 0, st>>>(bufs[r & 1], bufs[(r + 1) & 1], nr, N,
                                                  r ? &dsc->active[r - 1] : nullptr, &dsc->active[r],
                                                  &dsc->final_sel, (unsigned)((r + 1) & 1));
        EC_HIP(hipMemcpyAsync(&hsc, dsc, sizeof(Scalars), hipMemcpyDeviceToHost, st));
        EC_HIP(hipStreamSynchronize(st));
        unsigned int used = 1;
        for (int r = 0; r < rounds; r++)
            if (hsc.active[r]) used = r + 2;
        s->stats.rank_rounds = std::min<unsigned int>(used, rounds);
        if (hsc.active[rounds - 1] != 0) {
            set_error("ruler list ranking did not converge in %d rounds", rounds);
            s->events = saved_events;
            return EC_ERR_STATE;
        }
        fin = (hsc.final_sel & 1) ? s->st1.as<RJump>() : s->st0.as<RJump>();
        k_finalize<<<grid_for(N, B), B, 0, st>>>(s->upal.as<uint8_t>(), s->succ.as<unsigned int>(),
                                                s->rid.as<unsigned int>(), s->roff.as<unsigned int>(),
                                                s->rlist.as<unsigned int>(), fin, N, s->PK.as<unsigned int>(),
                                                s->RK.as<unsigned int>(), s->PL.as<unsigned int>(),
                                                s->PM.as<unsigned long long>());
        k_cycle_len<<<grid_for(nr, B), B, 0, st>>>(s->nextR.as<unsigned int>(), s->rlist.as<unsigned int>(), fin, nr,
                                                  s->PL.as<unsigned int>(), s->PM.as<unsigned long long>());
    }
    s->stats.n_rulers = nr;
    mark(s, 2 * EC_STAGE_RANK + 1);

    // ---- starts + order -------------------------------------------------------------------
    mark(s, 2 * EC_STAGE_STARTS);
    EC_CHECK(s->cidxOf.ensure(Nn * 4));
    EC_CHECK(s->skeys.ensure(Nn * 8));
    EC_CHECK(s->svals.ensure(Nn * 4));
    EC_CHECK(s->skeys2.ensure(Nn * 8));
    EC_CHECK(s->svals2.ensure(Nn * 4));
    EC_HIP(hipMemsetAsync(s->cidxOf.p, 0xFF, Nn * 4, st));
    if (U)
        k_starts<<<grid_for(N, B), B, 0, st>>>(s->upal.as<uint8_t>(), s->dfc.as<unsigned long long>(),
                                              s->dft.as<unsigned long long>(), s->PK.as<unsigned int>(),
                                              s->PM.as<unsigned long long>(), N, s->skeys.as<unsigned long long>(),
                                              s->svals.as<unsigned int>(), &dsc->nstarts);
    EC_HIP(hipMemcpyAsync(&hsc.nstarts, &dsc->nstarts, 4, hipMemcpyDeviceToHost, st));
    EC_HIP(hipStreamSynchronize(st));
    const unsigned int nc = hsc.nstarts;
    s->stats.n_contigs = nc;
    if (nc)
        EC_CHECK(sort_pairs(s, s->skeys.as<unsigned long long>(), s->skeys2.as<unsigned long long>(),
                            s->svals.as<unsigned int>(), s->svals2.as<unsigned int>(), nc));
    const unsigned int *sorted_nodes = s->svals2.as<unsigned int>();
    EC_CHECK(s->clen.ensure((size_t)(nc + 1) * 8));
    EC_CHECK(s->coff.ensure((size_t)(nc + 1) * 8));
    EC_HIP(hipMemsetAsync(s->clen.p, 0, (size_t)(nc + 1) * 8, st));
    if (nc) {
        k_contig_len<<<grid_for(nc, B), B, 0, st>>>(s->upal.as<uint8_t>(), s->PK.as<unsigned int>(),
                                                   s->RK.as<unsigned int>(), s->PL.as<unsigned int>(), sorted_nodes, nc,
                                                   k, s->cidxOf.as<unsigned int>(), s->clen.as<unsigned long long>());
    }
    EC_CHECK(scan_u64(s, s->clen.as<unsigned long long>(), s->coff.as<unsigned long long>(), nc + 1));
    s->h_coff.assign(nc + 1, 0);
    EC_HIP(hipMemcpyAsync(s->h_coff.data(), s->coff.p, (size_t)(nc + 1) * 8, hipMemcpyDeviceToHost, st));
    EC_HIP(hipStreamSynchronize(st));
    mark(s, 2 * EC_STAGE_STARTS + 1);
    const uint64_t nchars = s->h_coff[nc];
    s->stats.n_contig_chars = nchars;

    // ---- emit -----------------------------------------------------------------------------
    mark(s, 2 * EC_STAGE_EMIT);
    EC_CHECK(s->chars.ensure(std::max<size_t>(nchars, 1)));
    EC_CHECK(s->cfirst.ensure((size_t)std::max(nc, 1u) * 4));
    EC_CHECK(s->clast.ensure((size_t)std::max(nc, 1u) * 4));
    EC_CHECK(s->headOf.ensure(Nn * 4));
    EC_CHECK(s->tailOf.ensure(Nn * 4));
    EC_HIP(hipMemsetAsync(s->headOf.p, 0xFF, Nn * 4, st));
    EC_HIP(hipMemsetAsync(s->tailOf.p, 0xFF, Nn * 4, st));
    if (U)
        k_emit<<<grid_for(N, B), B, 0, st>>>(s->upal.as<uint8_t>(), s->PK.as<unsigned int>(), s->RK.as<unsigned int>(),
                                            s->PL.as<unsigned int>(), s->dkey.as<unsigned long long>(),
                                            s->cidxOf.as<unsigned int>(), sorted_nodes, s->coff.as<unsigned long long>(),
                                            N, k, s->chars.as<char>(), s->cfirst.as<unsigned int>(),
                                            s->clast.as<unsigned int>(), s->headOf.as<unsigned int>(),
                                            s->tailOf.as<unsigned int>());
    mark(s, 2 * EC_STAGE_EMIT + 1);

    // ---- GFA ------------------------------------------------------------------------------
    mark(s, 2 * EC_STAGE_GFA);
    EC_CHECK(s->lk.ensure((size_t)std::max(nc, 1u) * 16 * 8));
    EC_CHECK(s->lcnt.ensure((size_t)std::max(nc, 1u) * 2 * 4));
    if (nc)
        k_gfa<<<grid_for(nc, B), B, 0, st>>>(s->table.as<Slot>(), cap - 1, s->dkey.as<unsigned long long>(),
                                            s->upal.as<uint8_t>(), s->cfirst.as<unsigned int>(),
                                            s->clast.as<unsigned int>(), s->headOf.as<unsigned int>(),
                                            s->tailOf.as<unsigned int>(), nc, k, s->lk.as<long long>(),
                                            s->lcnt.as<unsigned int>());
    mark(s, 2 * EC_STAGE_GFA + 1);

    // ---- results to host --------------------------------------------------------------------
    s->h_chars.resize(nchars);
    std::vector<unsigned int> lcnt(2 * (size_t)nc);
    std::vector<long long> lk(16 * (size_t)nc);
    if (nchars) EC_HIP(hipMemcpyAsync(s->h_chars.data(), s->chars.p, nchars, hipMemcpyDeviceToHost, st));
    if (nc) {
        EC_HIP(hipMemcpyAsync(lcnt.data(), s->lcnt.p, lcnt.size() * 4, hipMemcpyDeviceToHost, st));
        EC_HIP(hipMemcpyAsync(lk.data(), s->lk.p, lk.size() * 8, hipMemcpyDeviceToHost, st));
    }
    EC_HIP(hipStreamSynchronize(st));
    s->h_loff.assign(2 * (size_t)nc + 1, 0);
    s->h_links.clear();
    for (size_t i = 0; i < 2 * (size_t)nc; i++) {
        for (unsigned j = 0; j < lcnt[i]; j++) s->h_links.push_back(lk[i * 8 + j]);
        s->h_loff[i + 1] = s->h_links.size();
    }
    s->stats.n_links = s->h_links.size();

    s->stats.n_dict = 2ull * U - hsc.npal;  // len(build()): palindromes have one entry

    if (timing) {
        for (int i = 0; i < EC_NSTAGES; i++) {
            float ms = 0;
            hipEventElapsedTime(&ms, s->ev[2 * i], s->ev[2 * i + 1]);
            s->stats.stage_ms[i] = ms;
        }
        float ms = 0;
        hipEventElapsedTime(&ms, s->ev[2 * EC_NSTAGES], s->ev[2 * EC_NSTAGES + 1]);
        s->stats.count_kernel_ms = ms;
    }
    s->events = saved_events || timing;
    s->have = true;
    return EC_OK;
}

}  // namespace

extern "C" {

int ec_session_create(ec_session **out, int device) {
    if (!out) {
        set_error("null out");
        return EC_ERR_ARG;
    }
    int n = 0;
    EC_HIP(hipGetDeviceCount(&n));
    if (device < 0 || device >= n) {
        set_error("device %d not in [0,%d)", device, n);
        return EC_ERR_ARG;
    }
    EC_HIP(hipSetDevice(device));
    ec_session *s = new ec_session();
    s->device = device;
    if (hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess) {
        delete s;
        set_error("hipStreamCreate failed");
        return EC_ERR_HIP;
    }
    s->own_stream = true;
    *out = s;
    return EC_OK;
}

int ec_session_set_stream(ec_session *s, void *hip_stream) {
    if (!s) return EC_ERR_ARG;
    if (s->own_stream && s->stream) hipStreamDestroy(s->stream);
    s->own_stream = false;
    s->stream = (hipStream_t)hip_stream;
    if (!hip_stream) {
        EC_HIP(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
        s->own_stream = true;
    }
    return EC_OK;
}

int ec_session_destroy(ec_session *s) {
    if (!s) return EC_OK;
    hipSetDevice(s->device);
    if (s->stream) hipStreamSynchronize(s->stream);
    DevBuf *all[] = {&s->h_reads, &s->h_offsets, &s->hll, &s->scal, &s->table, &s->dkey, &s->dcnt, &s->dfc, &s->dft,
                     &s->upal, &s->outdeg, &s->cand, &s->succ, &s->pred, &s->st0, &s->st1, &s->startOf, &s->skeys,
                     &s->svals, &s->skeys2, &s->svals2, &s->cidxOf, &s->clen, &s->coff, &s->chars, &s->cfirst,
                     &s->clast, &s->headOf, &s->tailOf, &s->lk, &s->lcnt, &s->tmp, &s->dchars, &s->dcounts,
                     &s->rid, &s->roff, &s->rlist, &s->nextR, &s->PK, &s->RK, &s->PL, &s->PM};
    for (auto *b : all) b->release();
    if (s->events)
        for (auto &e : s->ev) hipEventDestroy(e);
    if (s->own_stream && s->stream) hipStreamDestroy(s->stream);
    delete s;
    return EC_OK;
}

int ec_assemble_device(ec_session *s, const uint8_t *d_reads, const uint64_t *d_offsets, uint64_t nreads, int k,
                       int limit, unsigned flags) {
    if (!s || (!d_offsets)) {
        set_error("null session/offsets");
        return EC_ERR_ARG;
    }
    return assemble(s, d_reads, d_offsets, nreads, k, limit, flags);
}

int ec_assemble_host(ec_session *s, const uint8_t *reads, uint64_t nbytes, const uint64_t *offsets, uint64_t nreads,
                     int k, int limit, unsigned flags) {
    if (!s || !offsets || (nbytes && !reads)) {
        set_error("null argument");
        return EC_ERR_ARG;
    }
    if (offsets[nreads] > nbytes) {
        set_error("offsets[nreads]=%llu > nbytes=%llu", (unsigned long long)offsets[nreads], (unsigned long long)nbytes);
        return EC_ERR_ARG;
    }
    for (uint64_t i = 0; i < nreads; i++)
        if (offsets[i] > offsets[i + 1]) {
            set_error("offsets not monotone at %llu", (unsigned long long)i);
            return EC_ERR_ARG;
        }
    EC_HIP(hipSetDevice(s->device));
    EC_CHECK(s->h_reads.ensure(nbytes + 16));
    EC_CHECK(s->h_offsets.ensure((nreads + 1) * 8));
    if (nbytes) EC_HIP(hipMemcpyAsync(s->h_reads.p, reads, nbytes, hipMemcpyHostToDevice, s->stream));
    EC_HIP(hipMemcpyAsync(s->h_offsets.p, offsets, (nreads + 1) * 8, hipMemcpyHostToDevice, s->stream));
    return assemble(s, s->h_reads.as<uint8_t>(), s->h_offsets.as<uint64_t>(), nreads, k, limit, flags);
}

int ec_get_stats(ec_session *s, ec_stats *out) {
    if (!s || !out) return EC_ERR_ARG;
    if (!s->have) {
        set_error("no successful assembly in this session");
        return EC_ERR_STATE;
    }
    *out = s->stats;
    return EC_OK;
}

const char *ec_stage_name(int stage) {
    static const char *names[EC_NSTAGES] = {"prescan", "count", "compact", "links", "rank", "starts", "emit", "gfa"};
    return (stage >= 0 && stage < EC_NSTAGES) ? names[stage] : "?";
}

int ec_copy_contigs(ec_session *s, char *chars, uint64_t *offsets) {
    if (!s) return EC_ERR_ARG;
    if (!s->have) {
        set_error("no successful assembly in this session");
        return EC_ERR_STATE;
    }
    if (chars && !s->h_chars.empty()) memcpy(chars, s->h_chars.data(), s->h_chars.size());
    if (offsets) memcpy(offsets, s->h_coff.data(), s->h_coff.size() * 8);
    return EC_OK;
}

int ec_copy_links(ec_session *s, uint64_t *link_offsets, int64_t *links) {
    if (!s) return EC_ERR_ARG;
    if (!s->have) {
        set_error("no successful assembly in this session");
        return EC_ERR_STATE;
    }
    if (link_offsets) memcpy(link_offsets, s->h_loff.data(), s->h_loff.size() * 8);
    if (links && !s->h_links.empty()) memcpy(links, s->h_links.data(), s->h_links.size() * 8);
    return EC_OK;
}

int ec_copy_dict(ec_session *s, char *kmers, uint32_t *counts) {
    if (!s) return EC_ERR_ARG;
    if (!s->have || !s->want_dict) {
        set_error("ec_copy_dict needs a successful ec_assemble_* with EC_FLAG_WANT_DICT");
        return EC_ERR_STATE;
    }
    const unsigned int U = (unsigned int)s->stats.n_solid;
    const unsigned int N = 2 * U;
    const unsigned B = 256;
    if (!U) return EC_OK;
    hipStream_t st = s->stream;
    EC_HIP(hipSetDevice(s->device));
    Scalars *dsc = s->scal.as<Scalars>();
    EC_HIP(hipMemsetAsync(&dsc->ndict, 0, 4, st));
    k_dict_items<<<grid_for(N, B), B, 0, st>>>(s->upal.as<uint8_t>(), s->dfc.as<unsigned long long>(),
                                              s->dft.as<unsigned long long>(), N, s->skeys.as<unsigned long long>(),
                                              s->svals.as<unsigned int>(), &dsc->ndict);
    unsigned int nd = 0;
    EC_HIP(hipMemcpyAsync(&nd, &dsc->ndict, 4, hipMemcpyDeviceToHost, st));
    EC_HIP(hipStreamSynchronize(st));
    EC_CHECK(sort_pairs(s, s->skeys.as<unsigned long long>(), s->skeys2.as<unsigned long long>(),
                        s->svals.as<unsigned int>(), s->svals2.as<unsigned int>(), nd));
    EC_CHECK(s->dchars.ensure((size_t)nd * s->k));
    EC_CHECK(s->dcounts.ensure((size_t)nd * 4));
    k_dict_render<<<grid_for(nd, B), B, 0, st>>>(s->svals2.as<unsigned int>(), nd, s->dkey.as<unsigned long long>(),
                                                s->dcnt.as<unsigned int>(), s->k, s->dchars.as<char>(),
                                                s->dcounts.as<unsigned int>());
    if (kmers) EC_HIP(hipMemcpyAsync(kmers, s->dchars.p, (size_t)nd * s->k, hipMemcpyDeviceToHost, st));
    if (counts) EC_HIP(hipMemcpyAsync(counts, s->dcounts.p, (size_t)nd * 4, hipMemcpyDeviceToHost, st));
    EC_HIP(hipStreamSynchronize(st));
    return EC_OK;
}

}  // extern "C"
