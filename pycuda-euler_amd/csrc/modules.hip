// modules.hip -- per-module drop-ins for the reference's PyCUDA module functions (layer 2 of
// include/eulerhip.h).  Host buffers in / out, like the reference's drv.In / .get() round
// trips; every kernel restates the INTENDED semantics of the reference kernel it replaces
// (file:line cited), with the reference's out-of-bounds / race defects fixed and,
// where a caller may depend on it, a flag that reproduces the reference's behaviour.
#include "common.h"

#include <rocprim/rocprim.hpp>

#include <algorithm>
#include <vector>

namespace ec {

// reference codeF / codeR tables (src/pyencode.py:40-41), indexed by (c & 7)
__device__ inline uint32_t codeF(uint32_t c) { return (0x20031000u >> ((c & 7u) * 4)) & 0xFu; }
__device__ inline uint32_t codeR(uint32_t c) { return (0x10002030u >> ((c & 7u) * 4)) & 0xFu; }

// ---- E1 encodeLmerDevice (src/pyencode.py:43-74) --------------------------------------------
// lmer[p] = sum_i codeF(buf[p+i]) << 2(L-1-i): the first L bases of buf[p..], MSB first.
// Bytes past the end of the buffer read as 0 (the reference reads past the end).
__global__ void __launch_bounds__(256) k_encode_lmer(const uint8_t *buf, uint64_t n, uint32_t L, int rc,
                                                     unsigned long long *out) {
    __shared__ uint8_t tile[256 + 32];
    for (uint64_t b0 = (uint64_t)blockIdx.x * 256; b0 < n; b0 += (uint64_t)gridDim.x * 256) {
        __syncthreads();
        for (unsigned i = threadIdx.x; i < 256 + 32; i += blockDim.x) tile[i] = (b0 + i < n) ? buf[b0 + i] : 0;
        __syncthreads();
        const uint64_t p = b0 + threadIdx.x;
        if (p < n) {
            unsigned long long v = 0;
            if (!rc) {
                for (uint32_t i = 0; i < L; i++) v = (v << 2) | codeF(tile[threadIdx.x + i]);
            } else {  // encodeLmerComplementDevice intended (:199-203): sum codeR(c[p+i]) << 2i
                for (uint32_t i = 0; i < L; i++) v |= (unsigned long long)codeR(tile[threadIdx.x + i]) << (2 * i);
            }
            out[p] = v;
        }
    }
}

// ---- E2 computeKmerDevice (src/pyencode.py:107-133) ------------------------------------------
__global__ void __launch_bounds__(256) k_split(const unsigned long long *lmers, uint64_t n, unsigned long long mask,
                                               unsigned long long *pk, unsigned long long *sk) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < n; t += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned long long l = lmers[t];
        pk[t] = (l & (mask << 2)) >> 2;  // LMER_PREFIX
        sk[t] = l & mask;                // LMER_SUFFIX
    }
}

// ---- H1-H6 bucketed static hash (src/pygpuhash.py, src/pydebruijn.py:56-87) ------------------
constexpr uint32_t BUCKET_ITEMS = 520;  // MAX_BUCKET_ITEM (src/pygpuhash.py:14)

__host__ __device__ inline uint32_t hash_h(unsigned long long key, uint32_t nb) {
    return (uint32_t)(((0x01010101ull + 0x12345678ull * key) % 1900813ull) % nb);  // :32-35
}

// phase1 (:36-51): per-bucket counts
__global__ void __launch_bounds__(256) k_hash_count(const unsigned long long *keys, uint64_t n, uint32_t nb,
                                                    unsigned int *bsize) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < n; t += (uint64_t)gridDim.x * blockDim.x)
        atomicAdd(&bsize[hash_h(keys[t], nb)], 1u);
}

// copyToBucket (:94-126): scatter (key, input index) to the bucket's staging range
__global__ void __launch_bounds__(256) k_hash_scatter(const unsigned long long *keys, uint64_t n, uint32_t nb,
                                                      const unsigned long long *start, unsigned int *cursor,
                                                      unsigned long long *bk, unsigned int *bi) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < n; t += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t b = hash_h(keys[t], nb);
        const unsigned long long p = start[b] + atomicAdd(&cursor[b], 1u);
        bk[p] = keys[t];
        bi[p] = (unsigned int)t;
    }
}

// bucketSort (:186-231): TK[b*520 + rank] with rank = #{keys of the bucket < key}.  Equal
// keys share a rank as in the reference; the highest input index then wins (deterministic).
__global__ void __launch_bounds__(256) k_hash_bucket_sort(const unsigned long long *bk, const unsigned int *bi,
                                                          const unsigned long long *start, const unsigned int *bsize,
                                                          const unsigned int *vals, unsigned long long *TK,
                                                          unsigned int *TV) {
    __shared__ unsigned long long keys[BUCKET_ITEMS];
    __shared__ unsigned int idx[BUCKET_ITEMS];
    __shared__ unsigned int win[BUCKET_ITEMS];
    const uint32_t b = blockIdx.x;
    const unsigned int s = bsize[b];
    const unsigned long long o = start[b];
    for (unsigned i = threadIdx.x; i < s; i += blockDim.x) {
        keys[i] = bk[o + i];
        idx[i] = bi[o + i];
        win[i] = 0;
    }
    __syncthreads();
    for (unsigned i = threadIdx.x; i < s; i += blockDim.x) {
        unsigned int rank = 0;
        for (unsigned j = 0; j < s; j++) rank += keys[j] < keys[i];
        atomicMax(&win[rank], idx[i] + 1);
    }
    __syncthreads();
    for (unsigned i = threadIdx.x; i < s; i += blockDim.x) {
        unsigned int rank = 0;
        for (unsigned j = 0; j < s; j++) rank += keys[j] < keys[i];
        if (win[rank] == idx[i] + 1) {
            TK[(uint64_t)b * BUCKET_ITEMS + rank] = keys[i];
            TV[(uint64_t)b * BUCKET_ITEMS + rank] = vals[idx[i]];
        }
    }
}

// phase1 offsets, deterministic: position of the key among the keys of its bucket in input
// order (the reference's atomicInc order is arbitrary); bi = input indices sorted stably by bucket
__global__ void __launch_bounds__(256) k_hash_offsets(const unsigned int *sorted_idx, const unsigned int *sorted_b,
                                                      uint64_t n, const unsigned long long *start,
                                                      unsigned int *offset) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < n; t += (uint64_t)gridDim.x * blockDim.x)
        offset[sorted_idx[t]] = (unsigned int)(t - start[sorted_b[t]]);
}

__global__ void __launch_bounds__(256) k_hash_bucket_ids(const unsigned long long *keys, uint64_t n, uint32_t nb,
                                                         unsigned int *b, unsigned int *idx) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < n; t += (uint64_t)gridDim.x * blockDim.x) {
        b[t] = hash_h(keys[t], nb);
        idx[t] = (unsigned int)t;
    }
}

// copyToBucket with given offsets (:94-126)
__global__ void __launch_bounds__(256) k_hash_copy(const unsigned long long *keys, const unsigned int *vals,
                                                   const unsigned int *offset, uint64_t n, uint32_t nb,
                                                   const unsigned int *start, unsigned long long *bk, unsigned int *bv) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < n; t += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t p = (uint64_t)start[hash_h(keys[t], nb)] + offset[t];
        bk[p] = keys[t];
        bv[p] = vals[t];
    }
}

// getHashValue (src/pydebruijn.py:56-87): binary search in the key's bucket; miss = 0xFFFFFFFF
__device__ inline unsigned int hash_get(unsigned long long key, const unsigned long long *TK, const unsigned int *TV,
                                        const unsigned int *bsize, uint32_t nb) {
    const uint32_t b = hash_h(key, nb);
    unsigned int lo = 0, hi = bsize[b];
    const unsigned long long *row = TK + (uint64_t)b * BUCKET_ITEMS;
    while (lo < hi) {
        const unsigned int mid = lo + (hi - lo) / 2;
        if (row[mid] < key) lo = mid + 1;
        else hi = mid;
    }
    return (lo < bsize[b] && row[lo] == key) ? TV[(uint64_t)b * BUCKET_ITEMS + lo] : NONE32;
}

__global__ void __launch_bounds__(256) k_hash_lookup(const unsigned long long *TK, const unsigned int *TV,
                                                     const unsigned int *bsize, uint32_t nb,
                                                     const unsigned long long *keys, uint64_t n, unsigned int *out) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < n; t += (uint64_t)gridDim.x * blockDim.x)
        out[t] = hash_get(keys[t], TK, TV, bsize, nb);
}

// ---- G1-G4 de Bruijn graph (src/pydebruijn.py) -------------------------------------------
struct EulerVertex {  // src/pydebruijn.py:196-202 (24 B, packed like the numpy dtype)
    unsigned long long vid;
    unsigned int ep, ecount, lp, lcount;
};
struct EulerEdge {  // src/pydebruijn.py:344-350 (24 B)
    unsigned long long eid;
    unsigned int v1, v2, s, pad;
};
static_assert(sizeof(EulerVertex) == 24 && sizeof(EulerEdge) == 24, "euler structs");

struct HashView {
    const unsigned long long *TK;
    const unsigned int *TV, *bsize;
    uint32_t nb;
    __device__ inline unsigned int get(unsigned long long k) const { return hash_get(k, TK, TV, bsize, nb); }
};

// per l-mer: prefix / suffix vertex, first / last base (debruijnCount :89-145)
__device__ inline void lmer_geometry(unsigned long long lmer, unsigned long long mask, const HashView &h,
                                     unsigned int &pi, unsigned int &si, uint64_t &to, uint64_t &from) {
    const unsigned long long prefix = (lmer & (mask << 2)) >> 2;
    const unsigned long long suffix = lmer & mask;
    pi = h.get(prefix);
    si = h.get(suffix);
    const unsigned long long tTo = lmer & 3ull;
    const unsigned long long tFrom = (lmer >> __popcll(mask)) & 3ull;
    // the reference forms (prefixIndex << 2) in 32 bits: a miss (0xFFFFFFFF) lands far out
    to = (uint64_t)((pi << 2) & 0xFFFFFFFFu) + tTo;
    from = (uint64_t)((si << 2) & 0xFFFFFFFFu) + tFrom;
}

__global__ void __launch_bounds__(256) k_db_count(const unsigned long long *lk, const unsigned int *lv, uint64_t nl,
                                                  HashView h, unsigned long long mask, uint64_t size,
                                                  unsigned int *lcount, unsigned int *ecount) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < nl; t += (uint64_t)gridDim.x * blockDim.x) {
        unsigned int pi, si;
        uint64_t to, from;
        lmer_geometry(lk[t], mask, h, pi, si, to, from);
        if (to < size) lcount[to] = lv[t];
        if (from < size) ecount[from] = lv[t];
    }
}

// setupVertices (:259-295)
__global__ void __launch_bounds__(256) k_db_vertices(const unsigned long long *kk, uint64_t nk, HashView h,
                                                     const unsigned int *lcount, const unsigned int *lstart,
                                                     const unsigned int *ecount, const unsigned int *estart,
                                                     EulerVertex *ev) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < nk; t += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned long long key = kk[t];
        const unsigned int i = h.get(key);
        if (i < nk) {
            const uint64_t q = 4ull * i;
            EulerVertex v;
            v.vid = key;
            v.lp = lstart[q];
            v.lcount = lcount[q] + lcount[q + 1] + lcount[q + 2] + lcount[q + 3];
            v.ep = estart[q];
            v.ecount = ecount[q] + ecount[q + 1] + ecount[q + 2] + ecount[q + 3];
            ev[i] = v;
        }
    }
}

// setupEdges (:403-477).  Fixed bounds: the vertex slots are checked against 4V (the
// reference compares with lmerCount, :449, dropping most edges; EC_MOD_REF_BOUNDS
// reproduces that) and edges are written up to E = sum of multiplicities.
__global__ void __launch_bounds__(256) k_db_edges(const unsigned long long *lk, const unsigned int *lv,
                                                  const unsigned int *loffs, uint64_t nl, HashView h,
                                                  unsigned long long mask, uint64_t size, uint64_t E, int refb,
                                                  const unsigned int *lstart, const unsigned int *estart,
                                                  unsigned int *l, unsigned int *e, EulerEdge *ee) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < nl; t += (uint64_t)gridDim.x * blockDim.x) {
        unsigned int pi, si;
        uint64_t to, from;
        lmer_geometry(lk[t], mask, h, pi, si, to, from);
        const uint64_t bound = refb ? (nl < size ? nl : size) : size;  // never past lstart/estart
        if (!(to < bound && from < bound)) continue;
        unsigned int lo = lstart[to], eo = estart[from], off = loffs[t];
        if (refb && off >= nl) continue;
        for (unsigned int j = 0; j < lv[t]; j++) {
            if (off >= E) break;
            EulerEdge x;
            x.eid = off;
            x.v1 = pi;
            x.v2 = si;
            x.s = (unsigned int)E;
            x.pad = 0;
            ee[off] = x;
            if (lo < E) l[lo] = off;
            if (eo < E) e[eo] = off;
            lo++;
            eo++;
            off++;
        }
    }
}

// ---- C1 connected components (src/pycomponent.py:668-723) --------------------------------
// Vertex{vid, n1, n2}; edges i-n1, i-n2 for neighbours < n.  Fixpoint of min-label hooking +
// pointer jumping: D[i] = the smallest vertex index of i's component (the reference stops
// after one Shiloach-Vishkin iteration, :716).
struct Vtx {
    unsigned int vid, n1, n2;
};

__global__ void __launch_bounds__(256) k_cc_init(unsigned int *D, uint64_t n) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < n; t += (uint64_t)gridDim.x * blockDim.x)
        D[t] = (unsigned int)t;
}

__device__ inline unsigned int cc_find(const unsigned int *D, unsigned int x) {
    unsigned int p = D[x];
    while (true) {
        const unsigned int q = D[p];
        if (q == p) return p;
        p = q;
    }
}

__global__ void __launch_bounds__(256) k_cc_hook(const Vtx *v, uint64_t n, unsigned int *D, unsigned int *changed) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < n; t += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned int nb[2] = {v[t].n1, v[t].n2};
        for (int q = 0; q < 2; q++) {
            if (nb[q] >= n) continue;
            unsigned int a = cc_find(D, (unsigned int)t), b = cc_find(D, nb[q]);
            while (a != b) {  // lock-free union: link the larger root under the smaller
                const unsigned int hi = a > b ? a : b, lo = a < b ? a : b;
                if (atomicCAS(&D[hi], hi, lo) == hi) {
                    *changed = 1;
                    break;
                }
                a = cc_find(D, hi);
                b = cc_find(D, lo);
            }
        }
    }
}

__global__ void __launch_bounds__(256) k_cc_compress(unsigned int *D, uint64_t n) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < n; t += (uint64_t)gridDim.x * blockDim.x)
        D[t] = cc_find(D, D[t]);
}

// ---- T1-T3 Euler tour machinery (src/pyeulertour.py) -----------------------------------------
// assignSuccessor (:53-83)
__global__ void __launch_bounds__(256) k_assign_successor(const EulerVertex *ev, uint64_t vcount, const unsigned int *l,
                                                          const unsigned int *e, EulerEdge *ee, uint64_t E) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < vcount; t += (uint64_t)gridDim.x * blockDim.x) {
        const EulerVertex v = ev[t];
        for (unsigned int i = 0; i < v.ecount && i < v.lcount; i++) {
            const uint64_t ei = (uint64_t)v.ep + i, li = (uint64_t)v.lp + i;
            if (ei < E) {
                const unsigned int x = e[ei];
                if (li < E && x < E) ee[x].s = l[li];
            }
        }
    }
}

// constructSuccessorGraphP1/P2 (:133-144, :187-199)
__global__ void __launch_bounds__(256) k_succ_graph1(const EulerEdge *ee, uint64_t E, Vtx *v) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < E; t += (uint64_t)gridDim.x * blockDim.x) {
        Vtx x;
        x.vid = (unsigned int)ee[t].eid;
        x.n1 = ee[t].s;
        x.n2 = (unsigned int)E;
        v[t] = x;
    }
}
__global__ void __launch_bounds__(256) k_succ_graph2(Vtx *v, uint64_t E) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < E; t += (uint64_t)gridDim.x * blockDim.x)
        if (v[t].n1 < E) v[v[t].n1].n2 = v[t].vid;
}

// calculateCircuitGraphVertexData (:223-231)
__global__ void __launch_bounds__(256) k_circuit_mark(const unsigned int *D, uint64_t E, unsigned int *C) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < E; t += (uint64_t)gridDim.x * blockDim.x)
        C[D[t]] = 1;
}

// calculateCircuitGraphEdgeData (:331-371) / assignCircuitGraphEdgeData (:428-469): adjacent
// entering edges of a vertex that lie on different circuits form a circuit-graph edge
struct CircuitEdge {  // :420-427
    unsigned int ceid, e1, e2, c1, c2;
};

__global__ void __launch_bounds__(256) k_circuit_edges(const EulerVertex *ev, uint64_t vcount, const unsigned int *e,
                                                       const unsigned int *D, const unsigned int *map, uint64_t E,
                                                       unsigned int *slot, CircuitEdge *out) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < vcount; t += (uint64_t)gridDim.x * blockDim.x) {
        const EulerVertex v = ev[t];
        if (v.ecount == 0) continue;
        const uint64_t maxIndex = (uint64_t)v.ep + v.ecount - 1;
        for (uint64_t index = v.ep; index < maxIndex && index + 1 < E; index++) {
            if (!(e[index] < E && e[index + 1] < E)) continue;
            const unsigned int c1 = map[D[e[index]]], c2 = map[D[e[index + 1]]];
            if (c1 == c2) continue;
            CircuitEdge x;
            x.ceid = 0;  // never assigned by the reference kernel
            x.e1 = e[index];
            x.e2 = e[index + 1];
            x.c1 = min(c1, c2);
            x.c2 = max(c1, c2);
            // slot order is arbitrary (atomicDec in the reference); callers sort by (c1, c2) (:791)
            out[atomicAdd(slot, 1u)] = x;
        }
    }
}

// markSpanningEulerEdges (:613-632) and executeSwipe (:518-557)
// tree_first = 0: mark[min(e1, e2)] (:627); 1 (EC_MOD_TREE_MARKS): mark[e1], the first of the
// two consecutive entering edges the circuit-graph edge joins (e1 = e[i], e2 = e[i + 1],
// k_circuit_edges), which is the edge whose run the swipe rotates
__global__ void __launch_bounds__(256) k_mark_spanning(const CircuitEdge *cg, const unsigned int *tree, uint64_t nt,
                                                       uint64_t E, unsigned int *mark, int tree_first) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < nt; t += (uint64_t)gridDim.x * blockDim.x) {
        const CircuitEdge c = cg[tree[t]];
        const unsigned int m = tree_first ? c.e1 : min(c.e1, c.e2);
        if (m < E) mark[m] = 1;
    }
}

// the swipe body the reference comments out (:534-555): at every vertex, each run of marked
// entering edges e_t .. e_{j-1} (and the edge e_j that ends it) rotates its successors,
// s(e_i) = s(e_{i+1}), s(e_j) = old s(e_t) -- merging the circuits of e_t .. e_j into one
__global__ void __launch_bounds__(256) k_swipe(const EulerVertex *ev, uint64_t vcount, const unsigned int *e,
                                               EulerEdge *ee, const unsigned int *mark, uint64_t E) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < vcount; t += (uint64_t)gridDim.x * blockDim.x) {
        const EulerVertex v = ev[t];
        if (v.ecount == 0) continue;
        uint64_t index = v.ep;
        const uint64_t maxIndex = index + v.ecount - 1;
        if (maxIndex >= E) continue;
        while (index < maxIndex && ee[e[index]].eid < E) {
            if (mark[ee[e[index]].eid] == 1) {
                const uint64_t t0 = index;
                const unsigned int s = ee[e[index]].s;
                while (mark[ee[e[index]].eid] == 1 && index < maxIndex) {
                    ee[e[index]].s = ee[e[index + 1]].s;
                    index++;
                }
                if (t0 != index) ee[e[index]].s = s;
            }
            index++;
        }
    }
}

// identifyContigStart (:680-688); contigStart is u32 here (the reference passes u32 to an
// unsigned char* kernel)
__global__ void __launch_bounds__(256) k_contig_start(const EulerEdge *ee, uint64_t E, unsigned int *cs) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < E; t += (uint64_t)gridDim.x * blockDim.x)
        if (ee[t].s < E) cs[ee[t].s] = 0;
}


// ---- H0 readLmersKmersCuda host dedup, on the device (src/eulercuda.py:73-179) -------------
// streams: l-mers S[2p] = F[p], S[2p+1] = R[p] (:147-160); k-mers K[4p..4p+3] = pF, sF, pR, sR
// (:142-145).  unique_first() keeps each distinct key once, in order of first occurrence in
// the stream (= Python dict insertion order), with its multiplicity.
__global__ void __launch_bounds__(256) k_streams(const unsigned long long *F, const unsigned long long *R, uint64_t B,
                                                 unsigned long long mask, unsigned long long *S,
                                                 unsigned long long *K) {
    for (uint64_t p = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; p < B; p += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned long long f = F[p], r = R[p];
        S[2 * p] = f;
        S[2 * p + 1] = r;
        K[4 * p + 0] = (f & (mask << 2)) >> 2;
        K[4 * p + 1] = f & mask;
        K[4 * p + 2] = (r & (mask << 2)) >> 2;
        K[4 * p + 3] = r & mask;
    }
}

__global__ void __launch_bounds__(256) k_iota(unsigned int *x, uint64_t n) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < n; t += (uint64_t)gridDim.x * blockDim.x)
        x[t] = (unsigned int)t;
}

// segment heads of the sorted keys (zero keys excluded when skip_zero)
__global__ void __launch_bounds__(256) k_seg_heads(const unsigned long long *sk, uint64_t n, int skip_zero,
                                                   unsigned int *flag) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < n; t += (uint64_t)gridDim.x * blockDim.x)
        flag[t] = (t == 0 || sk[t] != sk[t - 1]) && !(skip_zero && sk[t] == 0ull);
}

__global__ void __launch_bounds__(256) k_seg_compact(const unsigned long long *sk, const unsigned int *si,
                                                     const unsigned int *flag, const unsigned int *pos, uint64_t n,
                                                     unsigned long long *uk, unsigned int *ufirst, unsigned int *ustart) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < n; t += (uint64_t)gridDim.x * blockDim.x)
        if (flag[t]) {
            const unsigned int j = pos[t];
            uk[j] = sk[t];
            ufirst[j] = si[t];  // the radix sort is stable: the head holds the first occurrence
            ustart[j] = (unsigned int)t;
        }
}

__global__ void __launch_bounds__(256) k_seg_emit(const unsigned int *order, const unsigned long long *uk,
                                                  const unsigned int *ustart, uint64_t nu, uint64_t n,
                                                  unsigned long long *out_k, unsigned int *out_c) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < nu; t += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned int j = order[t];
        out_k[t] = uk[j];
        if (out_c) out_c[t] = (unsigned int)((j + 1 < nu ? ustart[j + 1] : n) - ustart[j]);
    }
}

__global__ void __launch_bounds__(256) k_count_zero(const unsigned long long *x, uint64_t n, unsigned long long *cnt) {
    unsigned long long c = 0;
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < n; t += (uint64_t)gridDim.x * blockDim.x)
        c += x[t] == 0ull;
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(cnt, c);
}

// ---- T6 generatePartialContig walk, on the device (src/eulercuda.py:328-402) ----------------
// With an injective successor map the edges form disjoint paths and cycles.  The reference's
// first loop emits every path from its head (edges that are no one's successor) in head order,
// the second loop every cycle from its smallest edge, in that order.  Pointer jumping on the
// predecessor links gives (head, rank); cycles are found (pointer never reaches a head after
// ceil(log2 E) + 1 doublings), cut at their minimum edge and ranked again.
__global__ void __launch_bounds__(256) k_pw_pred(const EulerEdge *ee, uint64_t E, unsigned int *pred,
                                                 unsigned int *indeg) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < E; t += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned int s = ee[t].s;
        if (s < E) {
            pred[s] = (unsigned int)t;
            atomicAdd(&indeg[s], 1u);
        }
    }
}

__global__ void __launch_bounds__(256) k_pw_init(const unsigned int *pred, const unsigned int *mn_in, uint64_t E,
                                                 unsigned int *nxt, unsigned int *d, unsigned int *hd,
                                                 unsigned int *mn) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < E; t += (uint64_t)gridDim.x * blockDim.x) {
        unsigned int p = pred[t];
        if (mn_in && mn_in[t] == (unsigned int)t) p = NONE32;  // cut a cycle at its minimum edge
        nxt[t] = p;
        d[t] = p == NONE32 ? 0u : 1u;
        hd[t] = p == NONE32 ? (unsigned int)t : p;
        mn[t] = (unsigned int)t;
    }
}

__global__ void __launch_bounds__(256) k_pw_jump(const unsigned int *nxt, const unsigned int *d, const unsigned int *hd,
                                                 const unsigned int *mn, uint64_t E, unsigned int *nxt2,
                                                 unsigned int *d2, unsigned int *hd2, unsigned int *mn2) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < E; t += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned int q = nxt[t];
        if (q == NONE32) {
            nxt2[t] = q;
            d2[t] = d[t];
            hd2[t] = hd[t];
            mn2[t] = mn[t];
        } else {
            nxt2[t] = nxt[q];
            d2[t] = d[t] + d[q];
            hd2[t] = hd[q];
            mn2[t] = min(mn[t], mn[q]);
        }
    }
}

// cycle members keep a live pointer; their window minimum is the cycle minimum
__global__ void __launch_bounds__(256) k_pw_cycmin(const unsigned int *nxt, const unsigned int *mn, uint64_t E,
                                                   unsigned int *cmin) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < E; t += (uint64_t)gridDim.x * blockDim.x)
        cmin[t] = nxt[t] == NONE32 ? NONE32 : mn[t];
}

__global__ void __launch_bounds__(256) k_pw_keys(const unsigned int *cmin, const unsigned int *hd, const unsigned int *d,
                                                 uint64_t E, unsigned long long *key, unsigned int *val) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < E; t += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned long long cyc = cmin[t] != NONE32;
        key[t] = (cyc << 63) | ((unsigned long long)hd[t] << 32) | d[t];
        val[t] = (unsigned int)t;
    }
}

// chars contributed by the edge at sorted position j: its v1 (l-1)-mer, plus v2's when it ends the walk
__global__ void __launch_bounds__(256) k_pw_len(const unsigned long long *skey, uint64_t E, unsigned int km1,
                                                unsigned long long *len, unsigned int *start) {
    for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < E; j += (uint64_t)gridDim.x * blockDim.x) {
        const bool first = (unsigned int)skey[j] == 0u;
        const bool last = j + 1 == E || (unsigned int)skey[j + 1] == 0u;
        len[j] = (unsigned long long)km1 * (last ? 2 : 1);
        start[j] = first;
    }
}

__device__ inline void put_kmer(char *out, unsigned long long vid, unsigned int km1) {
    for (unsigned int t = 0; t < km1; t++) out[t] = "ACGT"[(vid >> (2 * (km1 - 1 - t))) & 3ull];  // getString :314-320
}

__global__ void __launch_bounds__(256) k_pw_emit(const unsigned long long *skey, const unsigned int *sval,
                                                 const unsigned long long *pos, const unsigned int *cidx, uint64_t E,
                                                 const EulerEdge *ee, const EulerVertex *ev, uint64_t vcount,
                                                 unsigned int km1, char *chars, unsigned long long *coff,
                                                 unsigned int *bad) {
    for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < E; j += (uint64_t)gridDim.x * blockDim.x) {
        const EulerEdge x = ee[sval[j]];
        if (x.v1 >= vcount || x.v2 >= vcount) {
            atomicOr(bad, 1u);
            continue;
        }
        put_kmer(chars + pos[j], ev[x.v1].vid, km1);
        const bool last = j + 1 == E || (unsigned int)skey[j + 1] == 0u;
        if (last) put_kmer(chars + pos[j] + km1, ev[x.v2].vid, km1);
        if ((unsigned int)skey[j] == 0u) coff[cidx[j] - 1] = pos[j];
    }
}

// ---- host helpers ---------------------------------------------------------------------------
struct Dev {
    void *p = nullptr;
    explicit Dev(size_t bytes) {
        if (hipMalloc(&p, std::max<size_t>(bytes, 16)) != hipSuccess) p = nullptr;
    }
    ~Dev() {
        if (p) (void)hipFree(p);
    }
    template <typename T>
    T *as() const { return reinterpret_cast<T *>(p); }
    Dev(const Dev &) = delete;
};

#define EC_DEV(name, bytes)                                   \
    Dev name(bytes);                                          \
    if (!name.p) {                                            \
        set_error("hipMalloc(%zu) failed", (size_t)(bytes)); \
        return EC_ERR_NOMEM;                                  \
    }

int exscan_u32(const unsigned int *in, unsigned int *out, size_t n) {
    size_t bytes = 0;
    EC_HIP(rocprim::exclusive_scan(nullptr, bytes, in, out, 0u, n, rocprim::plus<unsigned int>(), (hipStream_t)0));
    EC_DEV(tmp, bytes);
    EC_HIP(rocprim::exclusive_scan(tmp.p, bytes, in, out, 0u, n, rocprim::plus<unsigned int>(), (hipStream_t)0));
    return EC_OK;
}

int exscan_u64(const unsigned int *in, unsigned long long *out, size_t n) {
    size_t bytes = 0;
    EC_HIP(rocprim::exclusive_scan(nullptr, bytes, in, out, 0ull, n, rocprim::plus<unsigned long long>(), (hipStream_t)0));
    EC_DEV(tmp, bytes);
    EC_HIP(rocprim::exclusive_scan(tmp.p, bytes, in, out, 0ull, n, rocprim::plus<unsigned long long>(), (hipStream_t)0));
    return EC_OK;
}

int components_dev(const Vtx *v, uint64_t n, unsigned int *D) {
    if (!n) return EC_OK;
    EC_DEV(flag, 4);
    k_cc_init<<<grid_for(n, 256), 256>>>(D, n);
    for (int it = 0; it < 64; it++) {
        EC_HIP(hipMemset(flag.p, 0, 4));
        k_cc_hook<<<grid_for(n, 256), 256>>>(v, n, D, flag.as<unsigned int>());
        k_cc_compress<<<grid_for(n, 256), 256>>>(D, n);
        unsigned int h = 0;
        EC_HIP(hipMemcpy(&h, flag.p, 4, hipMemcpyDeviceToHost));
        if (!h) return EC_OK;
    }
    set_error("components did not converge");
    return EC_ERR_STATE;
}

}  // namespace ec

using namespace ec;

// a user-supplied bucket table must keep every bucket inside its 520 slots (hash_get reads
// TK[b*520 .. b*520 + size[b]))
static int check_table(const uint32_t *bucket_size, uint32_t nb) {
    for (uint32_t b = 0; b < nb; b++)
        if (bucket_size[b] > BUCKET_ITEMS) {
            set_error("bucketSize[%u] = %u > MAX_BUCKET_ITEM=520", b, bucket_size[b]);
            return EC_ERR_ARG;
        }
    return EC_OK;
}

extern "C" {

static int encode_common(const uint8_t *buf, uint64_t n, uint32_t L, uint64_t *out, int rc) {
    if ((n && (!buf || !out)) || L < 1 || L > 32) {
        set_error("bad arguments (L=%u must be in [1,32])", L);
        return EC_ERR_ARG;
    }
    if (!n) return EC_OK;
    EC_DEV(db, n);
    EC_DEV(dout, n * 8);
    EC_HIP(hipMemcpy(db.p, buf, n, hipMemcpyHostToDevice));
    k_encode_lmer<<<grid_for(n, 256, 65535), 256>>>(db.as<uint8_t>(), n, L, rc, dout.as<unsigned long long>());
    EC_HIP(hipMemcpy(out, dout.p, n * 8, hipMemcpyDeviceToHost));
    return EC_OK;
}

int ec_encode_lmers(const uint8_t *buf, uint64_t n, uint32_t L, uint64_t *out) { return encode_common(buf, n, L, out, 0); }

int ec_encode_lmers_rc(const uint8_t *buf, uint64_t n, uint32_t L, uint64_t *out) {
    return encode_common(buf, n, L, out, 1);
}

int ec_split_kmers(const uint64_t *lmers, uint64_t n, uint64_t mask, uint64_t *pk, uint64_t *sk) {
    if (n && (!lmers || !pk || !sk)) {
        set_error("null argument");
        return EC_ERR_ARG;
    }
    if (!n) return EC_OK;
    EC_DEV(dl, n * 8);
    EC_DEV(dp, n * 8);
    EC_DEV(ds, n * 8);
    EC_HIP(hipMemcpy(dl.p, lmers, n * 8, hipMemcpyHostToDevice));
    k_split<<<grid_for(n, 256), 256>>>(dl.as<unsigned long long>(), n, mask, dp.as<unsigned long long>(),
                                      ds.as<unsigned long long>());
    EC_HIP(hipMemcpy(pk, dp.p, n * 8, hipMemcpyDeviceToHost));
    EC_HIP(hipMemcpy(sk, ds.p, n * 8, hipMemcpyDeviceToHost));
    return EC_OK;
}

uint32_t ec_hash_bucket_count(uint64_t n) { return (uint32_t)(n / 409 + 1); }  // src/pygpuhash.py:273

int ec_hash_build(const uint64_t *keys, const uint32_t *vals, uint64_t n, uint32_t nb, unsigned flags, uint64_t *TK,
                  uint32_t *TV, uint32_t *bucket_size) {
    if ((n && (!keys || !vals)) || !TK || !TV || !bucket_size) {
        set_error("null argument");
        return EC_ERR_ARG;
    }
    if (!nb) nb = ec_hash_bucket_count(n);
    // phase1 / copyToBucket launch floor(n/1024) blocks of 1024 threads (:57-61, :143-147)
    uint64_t used = n;
    if ((flags & EC_MOD_TAIL_DROP) && n >= 1024) used = (n / 1024) * 1024;
    const uint64_t slots = (uint64_t)nb * BUCKET_ITEMS;
    EC_DEV(dk, used * 8);
    EC_DEV(dv, n * 4);
    EC_DEV(dsz, nb * 4ull);
    EC_DEV(dcur, nb * 4ull);
    EC_DEV(dstart, (nb + 1) * 8ull);
    EC_DEV(dbk, used * 8);
    EC_DEV(dbi, used * 4);
    EC_DEV(dTK, slots * 8);
    EC_DEV(dTV, slots * 4);
    if (used) EC_HIP(hipMemcpy(dk.p, keys, used * 8, hipMemcpyHostToDevice));
    if (n) EC_HIP(hipMemcpy(dv.p, vals, n * 4, hipMemcpyHostToDevice));
    EC_HIP(hipMemset(dsz.p, 0, nb * 4ull));
    EC_HIP(hipMemset(dcur.p, 0, nb * 4ull));
    EC_HIP(hipMemset(dTK.p, 0, slots * 8));
    EC_HIP(hipMemset(dTV.p, 0, slots * 4));
    if (used) k_hash_count<<<grid_for(used, 256), 256>>>(dk.as<unsigned long long>(), used, nb, dsz.as<unsigned int>());
    std::vector<uint32_t> hsz(nb);
    EC_HIP(hipMemcpy(hsz.data(), dsz.p, nb * 4ull, hipMemcpyDeviceToHost));
    for (uint32_t b = 0; b < nb; b++)
        if (hsz[b] > BUCKET_ITEMS) {
            set_error("bucket %u holds %u keys > MAX_BUCKET_ITEM=520 (the reference would overrun)", b, hsz[b]);
            return EC_ERR_CAPACITY;
        }
    EC_CHECK(exscan_u64(dsz.as<unsigned int>(), dstart.as<unsigned long long>(), nb));
    if (used) {
        k_hash_scatter<<<grid_for(used, 256), 256>>>(dk.as<unsigned long long>(), used, nb,
                                                    dstart.as<unsigned long long>(), dcur.as<unsigned int>(),
                                                    dbk.as<unsigned long long>(), dbi.as<unsigned int>());
        k_hash_bucket_sort<<<nb, 256>>>(dbk.as<unsigned long long>(), dbi.as<unsigned int>(),
                                        dstart.as<unsigned long long>(), dsz.as<unsigned int>(), dv.as<unsigned int>(),
                                        dTK.as<unsigned long long>(), dTV.as<unsigned int>());
    }
    EC_HIP(hipMemcpy(TK, dTK.p, slots * 8, hipMemcpyDeviceToHost));
    EC_HIP(hipMemcpy(TV, dTV.p, slots * 4, hipMemcpyDeviceToHost));
    memcpy(bucket_size, hsz.data(), nb * 4ull);
    return EC_OK;
}

int ec_hash_lookup(const uint64_t *TK, const uint32_t *TV, const uint32_t *bucket_size, uint32_t nb,
                   const uint64_t *keys, uint64_t n, uint32_t *out) {
    if (!TK || !TV || !bucket_size || !nb || (n && (!keys || !out))) {
        set_error("bad arguments");
        return EC_ERR_ARG;
    }
    EC_CHECK(check_table(bucket_size, nb));
    if (!n) return EC_OK;
    const uint64_t slots = (uint64_t)nb * BUCKET_ITEMS;
    EC_DEV(dTK, slots * 8);
    EC_DEV(dTV, slots * 4);
    EC_DEV(dsz, nb * 4ull);
    EC_DEV(dk, n * 8);
    EC_DEV(dout, n * 4);
    EC_HIP(hipMemcpy(dTK.p, TK, slots * 8, hipMemcpyHostToDevice));
    EC_HIP(hipMemcpy(dTV.p, TV, slots * 4, hipMemcpyHostToDevice));
    EC_HIP(hipMemcpy(dsz.p, bucket_size, nb * 4ull, hipMemcpyHostToDevice));
    EC_HIP(hipMemcpy(dk.p, keys, n * 8, hipMemcpyHostToDevice));
    k_hash_lookup<<<grid_for(n, 256), 256>>>(dTK.as<unsigned long long>(), dTV.as<unsigned int>(),
                                            dsz.as<unsigned int>(), nb, dk.as<unsigned long long>(), n,
                                            dout.as<unsigned int>());
    EC_HIP(hipMemcpy(out, dout.p, n * 4, hipMemcpyDeviceToHost));
    return EC_OK;
}

int ec_debruijn_build(const uint64_t *lmer_keys, const uint32_t *lmer_values, uint64_t nl, const uint64_t *kmer_keys,
                      uint64_t nk, uint32_t l, const uint64_t *TK, const uint32_t *TV, const uint32_t *bucket_size,
                      uint32_t nb, unsigned flags, void *ev_out, void *ee_out, uint32_t *l_out, uint32_t *e_out,
                      uint64_t *edge_count) {
    if (l < 2 || l > 32 || !TK || !TV || !bucket_size || !nb || !edge_count || (nl && (!lmer_keys || !lmer_values)) ||
        (nk && (!kmer_keys || !ev_out))) {
        set_error("bad arguments (l=%u must be in [2,32])", l);
        return EC_ERR_ARG;
    }
    EC_CHECK(check_table(bucket_size, nb));
    uint64_t E = 0;
    for (uint64_t i = 0; i < nl; i++) E += lmer_values[i];
    *edge_count = E;
    if (!ee_out && E) return EC_OK;  // sizing call
    const unsigned long long mask = kmask64((int)l - 1);  // valid_bitmask: 2(l-1) ones (:526-529)
    const uint64_t size = 4 * nk;
    const uint64_t slots = (uint64_t)nb * BUCKET_ITEMS;
    EC_DEV(dTK, slots * 8);
    EC_DEV(dTV, slots * 4);
    EC_DEV(dsz, nb * 4ull);
    EC_DEV(dlk, nl * 8);
    EC_DEV(dlv, nl * 4);
    EC_DEV(dlo, nl * 4);
    EC_DEV(dkk, nk * 8);
    EC_DEV(dlc, size * 4);
    EC_DEV(dec, size * 4);
    EC_DEV(dls, size * 4);
    EC_DEV(des, size * 4);
    EC_DEV(dev, nk * sizeof(EulerVertex));
    EC_DEV(dee, E * sizeof(EulerEdge));
    EC_DEV(dl, E * 4);
    EC_DEV(de, E * 4);
    EC_HIP(hipMemcpy(dTK.p, TK, slots * 8, hipMemcpyHostToDevice));
    EC_HIP(hipMemcpy(dTV.p, TV, slots * 4, hipMemcpyHostToDevice));
    EC_HIP(hipMemcpy(dsz.p, bucket_size, nb * 4ull, hipMemcpyHostToDevice));
    if (nl) {
        EC_HIP(hipMemcpy(dlk.p, lmer_keys, nl * 8, hipMemcpyHostToDevice));
        EC_HIP(hipMemcpy(dlv.p, lmer_values, nl * 4, hipMemcpyHostToDevice));
    }
    if (nk) EC_HIP(hipMemcpy(dkk.p, kmer_keys, nk * 8, hipMemcpyHostToDevice));
    EC_HIP(hipMemset(dlc.p, 0, std::max<uint64_t>(size, 1) * 4));
    EC_HIP(hipMemset(dec.p, 0, std::max<uint64_t>(size, 1) * 4));
    EC_HIP(hipMemset(dev.p, 0, std::max<uint64_t>(nk, 1) * sizeof(EulerVertex)));
    EC_HIP(hipMemset(dee.p, 0, std::max<uint64_t>(E, 1) * sizeof(EulerEdge)));
    EC_HIP(hipMemset(dl.p, 0, std::max<uint64_t>(E, 1) * 4));
    EC_HIP(hipMemset(de.p, 0, std::max<uint64_t>(E, 1) * 4));
    const HashView h{dTK.as<unsigned long long>(), dTV.as<unsigned int>(), dsz.as<unsigned int>(), nb};
    if (nl)
        k_db_count<<<grid_for(nl, 256), 256>>>(dlk.as<unsigned long long>(), dlv.as<unsigned int>(), nl, h, mask, size,
                                              dlc.as<unsigned int>(), dec.as<unsigned int>());
    if (size) {
        EC_CHECK(exscan_u32(dlc.as<unsigned int>(), dls.as<unsigned int>(), size));
        EC_CHECK(exscan_u32(dec.as<unsigned int>(), des.as<unsigned int>(), size));
    }
    if (nl) EC_CHECK(exscan_u32(dlv.as<unsigned int>(), dlo.as<unsigned int>(), nl));
    if (nk)
        k_db_vertices<<<grid_for(nk, 256), 256>>>(dkk.as<unsigned long long>(), nk, h, dlc.as<unsigned int>(),
                                                 dls.as<unsigned int>(), dec.as<unsigned int>(), des.as<unsigned int>(),
                                                 dev.as<EulerVertex>());
    if (nl)
        k_db_edges<<<grid_for(nl, 256), 256>>>(dlk.as<unsigned long long>(), dlv.as<unsigned int>(),
                                              dlo.as<unsigned int>(), nl, h, mask, size, E,
                                              (flags & EC_MOD_REF_BOUNDS) ? 1 : 0, dls.as<unsigned int>(),
                                              des.as<unsigned int>(), dl.as<unsigned int>(), de.as<unsigned int>(),
                                              dee.as<EulerEdge>());
    if (nk) EC_HIP(hipMemcpy(ev_out, dev.p, nk * sizeof(EulerVertex), hipMemcpyDeviceToHost));
    if (E) {
        EC_HIP(hipMemcpy(ee_out, dee.p, E * sizeof(EulerEdge), hipMemcpyDeviceToHost));
        if (l_out) EC_HIP(hipMemcpy(l_out, dl.p, E * 4, hipMemcpyDeviceToHost));
        if (e_out) EC_HIP(hipMemcpy(e_out, de.p, E * 4, hipMemcpyDeviceToHost));
    }
    return EC_OK;
}

int ec_components(const void *vertices, uint64_t n, uint32_t *D) {
    if (n && (!vertices || !D)) {
        set_error("null argument");
        return EC_ERR_ARG;
    }
    if (!n) return EC_OK;
    EC_DEV(dv, n * sizeof(Vtx));
    EC_DEV(dD, n * 4);
    EC_HIP(hipMemcpy(dv.p, vertices, n * sizeof(Vtx), hipMemcpyHostToDevice));
    EC_CHECK(components_dev(dv.as<Vtx>(), n, dD.as<unsigned int>()));
    EC_HIP(hipMemcpy(D, dD.p, n * 4, hipMemcpyDeviceToHost));
    return EC_OK;
}

int ec_find_euler(const void *ev, uint64_t vcount, const uint32_t *l, const uint32_t *e, void *ee, uint64_t E,
                  void *cg_edges, uint64_t *cg_edge_count, uint32_t *cg_vertex_count) {
    if (!cg_edge_count || !cg_vertex_count || (vcount && !ev) || (E && (!l || !e || !ee || !cg_edges))) {
        set_error("null argument");
        return EC_ERR_ARG;
    }
    *cg_edge_count = 0;
    *cg_vertex_count = 0;
    if (!E) return EC_OK;
    EC_DEV(dev, vcount * sizeof(EulerVertex));
    EC_DEV(dl, E * 4);
    EC_DEV(de, E * 4);
    EC_DEV(dee, E * sizeof(EulerEdge));
    EC_DEV(dv, E * sizeof(Vtx));
    EC_DEV(dD, E * 4);
    EC_DEV(dC, E * 4);
    EC_DEV(dmap, E * 4);
    EC_DEV(dcnt, E * 4);
    EC_DEV(dcg, E * sizeof(CircuitEdge));
    if (vcount) EC_HIP(hipMemcpy(dev.p, ev, vcount * sizeof(EulerVertex), hipMemcpyHostToDevice));
    EC_HIP(hipMemcpy(dl.p, l, E * 4, hipMemcpyHostToDevice));
    EC_HIP(hipMemcpy(de.p, e, E * 4, hipMemcpyHostToDevice));
    EC_HIP(hipMemcpy(dee.p, ee, E * sizeof(EulerEdge), hipMemcpyHostToDevice));
    if (vcount)
        k_assign_successor<<<grid_for(vcount, 256), 256>>>(dev.as<EulerVertex>(), vcount, dl.as<unsigned int>(),
                                                          de.as<unsigned int>(), dee.as<EulerEdge>(), E);
    k_succ_graph1<<<grid_for(E, 256), 256>>>(dee.as<EulerEdge>(), E, dv.as<Vtx>());
    k_succ_graph2<<<grid_for(E, 256), 256>>>(dv.as<Vtx>(), E);
    EC_CHECK(components_dev(dv.as<Vtx>(), E, dD.as<unsigned int>()));
    EC_HIP(hipMemset(dC.p, 0, E * 4));
    k_circuit_mark<<<grid_for(E, 256), 256>>>(dD.as<unsigned int>(), E, dC.as<unsigned int>());
    EC_CHECK(exscan_u32(dC.as<unsigned int>(), dmap.as<unsigned int>(), E));
    uint32_t last[2];
    EC_HIP(hipMemcpy(&last[0], dmap.as<unsigned int>() + (E - 1), 4, hipMemcpyDeviceToHost));
    EC_HIP(hipMemcpy(&last[1], dC.as<unsigned int>() + (E - 1), 4, hipMemcpyDeviceToHost));
    const uint32_t cgV = last[0] + last[1];
    *cg_vertex_count = cgV;
    EC_HIP(hipMemcpy(ee, dee.p, E * sizeof(EulerEdge), hipMemcpyDeviceToHost));  // successors, in place
    if (cgV <= 1 || !vcount) return EC_OK;
    EC_HIP(hipMemset(dcnt.p, 0, 4));
    k_circuit_edges<<<grid_for(vcount, 256), 256>>>(dev.as<EulerVertex>(), vcount, de.as<unsigned int>(),
                                                   dD.as<unsigned int>(), dmap.as<unsigned int>(), E,
                                                   dcnt.as<unsigned int>(), dcg.as<CircuitEdge>());
    uint32_t total = 0;
    EC_HIP(hipMemcpy(&total, dcnt.p, 4, hipMemcpyDeviceToHost));
    *cg_edge_count = total;
    if (total) EC_HIP(hipMemcpy(cg_edges, dcg.p, total * sizeof(CircuitEdge), hipMemcpyDeviceToHost));
    return EC_OK;
}

int ec_execute_swipe(const void *ev, uint64_t vcount, const uint32_t *e, void *ee, uint64_t E, const void *cg_edges,
                     uint64_t cg_edge_count, const uint32_t *tree, uint64_t tree_count, unsigned flags, uint32_t *mark_out) {
    if ((E && (!e || !ee)) || (vcount && !ev) || (tree_count && (!tree || !cg_edges))) {
        set_error("null argument");
        return EC_ERR_ARG;
    }
    if (!E) return EC_OK;
    const EulerEdge *hee = static_cast<const EulerEdge *>(ee);
    for (uint64_t i = 0; i < E; i++)
        if (e[i] >= E || hee[i].eid >= E) {
            set_error("e[%llu] = %u / ee[%llu].eid out of range (E = %llu)", (unsigned long long)i, e[i],
                      (unsigned long long)i, (unsigned long long)E);
            return EC_ERR_ARG;
        }
    if (flags & EC_MOD_SWIPE) {  // each vertex rewrites its own entering edges: e must be a permutation
        std::vector<uint8_t> seen(E, 0);
        for (uint64_t i = 0; i < E; i++) {
            if (seen[e[i]]) {
                set_error("swipe needs e to be a permutation of the edges (edge %u listed twice)", e[i]);
                return EC_ERR_ARG;
            }
            seen[e[i]] = 1;
        }
    }
    for (uint64_t i = 0; i < tree_count; i++)
        if (tree[i] >= cg_edge_count) {
            set_error("tree[%llu] = %u is not a circuit-graph edge index", (unsigned long long)i, tree[i]);
            return EC_ERR_ARG;
        }
    EC_DEV(dev, vcount * sizeof(EulerVertex));
    EC_DEV(de, E * 4);
    EC_DEV(dee, E * sizeof(EulerEdge));
    EC_DEV(dcg, cg_edge_count * sizeof(CircuitEdge));
    EC_DEV(dt, tree_count * 4);
    EC_DEV(dm, E * 4);
    if (vcount) EC_HIP(hipMemcpy(dev.p, ev, vcount * sizeof(EulerVertex), hipMemcpyHostToDevice));
    EC_HIP(hipMemcpy(de.p, e, E * 4, hipMemcpyHostToDevice));
    EC_HIP(hipMemcpy(dee.p, ee, E * sizeof(EulerEdge), hipMemcpyHostToDevice));
    if (cg_edge_count) EC_HIP(hipMemcpy(dcg.p, cg_edges, cg_edge_count * sizeof(CircuitEdge), hipMemcpyHostToDevice));
    if (tree_count) EC_HIP(hipMemcpy(dt.p, tree, tree_count * 4, hipMemcpyHostToDevice));
    // mark starts as all ones (src/pyeulertour.py:659) -- or all zeros with EC_MOD_TREE_MARKS, so
    // only the spanning tree's edges rotate and each component's circuits merge into one tour
    std::vector<uint32_t> init(E, (flags & EC_MOD_TREE_MARKS) ? 0u : 1u);
    EC_HIP(hipMemcpy(dm.p, init.data(), E * 4, hipMemcpyHostToDevice));
    if (tree_count)
        k_mark_spanning<<<grid_for(tree_count, 256), 256>>>(dcg.as<CircuitEdge>(), dt.as<unsigned int>(), tree_count, E,
                                                           dm.as<unsigned int>(), (flags & EC_MOD_TREE_MARKS) ? 1 : 0);
    if ((flags & EC_MOD_SWIPE) && vcount)
        k_swipe<<<grid_for(vcount, 256), 256>>>(dev.as<EulerVertex>(), vcount, de.as<unsigned int>(),
                                               dee.as<EulerEdge>(), dm.as<unsigned int>(), E);
    EC_HIP(hipMemcpy(ee, dee.p, E * sizeof(EulerEdge), hipMemcpyDeviceToHost));
    if (mark_out) EC_HIP(hipMemcpy(mark_out, dm.p, E * 4, hipMemcpyDeviceToHost));
    return EC_OK;
}

int ec_identify_contig_start(const void *ee, uint64_t E, uint32_t *contig_start) {
    if (E && (!ee || !contig_start)) {
        set_error("null argument");
        return EC_ERR_ARG;
    }
    if (!E) return EC_OK;
    EC_DEV(dee, E * sizeof(EulerEdge));
    EC_DEV(dcs, E * 4);
    EC_HIP(hipMemcpy(dee.p, ee, E * sizeof(EulerEdge), hipMemcpyHostToDevice));
    EC_HIP(hipMemcpy(dcs.p, contig_start, E * 4, hipMemcpyHostToDevice));
    k_contig_start<<<grid_for(E, 256), 256>>>(dee.as<EulerEdge>(), E, dcs.as<unsigned int>());
    EC_HIP(hipMemcpy(contig_start, dcs.p, E * 4, hipMemcpyDeviceToHost));
    return EC_OK;
}

// ---- T4 findSpanningTree (src/eulercuda.py:266-305) -----------------------------------------
// The reference asks graph_tool for a minimum spanning tree of the circuit graph with unit
// weights (Kruskal); the result here is the forest Kruskal takes in edge-index order, i.e. the
// minimum spanning forest for weights = edge index -- unique, since those weights are distinct,
// so Boruvka rounds find it in parallel: every component picks its lowest-index outgoing edge,
// components hook along them (of a mutual pick, the larger root hooks to the smaller), then
// every vertex chases its new root.  Each round at least halves the components.
__global__ void __launch_bounds__(256) k_sf_best(const CircuitEdge *cg, uint64_t E, const unsigned int *comp,
                                                 unsigned int *best, unsigned int *any) {
    for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < E; j += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned int a = comp[cg[j].c1], b = comp[cg[j].c2];
        if (a != b) {
            atomicMin(&best[a], (unsigned int)j);
            atomicMin(&best[b], (unsigned int)j);
            *any = 1u;
        }
    }
}
__global__ void __launch_bounds__(256) k_sf_hook(const CircuitEdge *cg, uint64_t n, const unsigned int *comp,
                                                 const unsigned int *best, unsigned int *nxt, uint8_t *intree) {
    for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < n; r += (uint64_t)gridDim.x * blockDim.x) {
        nxt[r] = comp[r];
        if (comp[r] != r || best[r] == NONE32) continue;
        const unsigned int j = best[r];
        const unsigned int a = comp[cg[j].c1], b = comp[cg[j].c2];
        const unsigned int o = a == (unsigned int)r ? b : a;
        intree[j] = 1;
        if (best[o] == j && o > (unsigned int)r) continue;  // mutual pick: the larger root hooks
        nxt[r] = o;
    }
}
// the hooks form trees whose roots point to themselves, but not shallow ones: on a path whose
// edges are sorted by (c1, c2) every vertex hooks to its neighbour, one chain of length n.
// Pointer jumping (nxt[v] = nxt[nxt[v]], in place: a racing read only sees a pointer further up
// the same tree) reaches every root in ceil(log2(depth)) launches.
__global__ void __launch_bounds__(256) k_sf_jump(uint64_t n, unsigned int *nxt, unsigned int *changed) {
    bool ch = false;
    for (uint64_t v = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; v < n; v += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned int p = nxt[v], q = nxt[p];
        if (p != q) {
            nxt[v] = q;
            ch = true;
        }
    }
    if (__any(ch) && (threadIdx.x & 63) == 0) *changed = 1u;
}
__global__ void __launch_bounds__(256) k_sf_settle(uint64_t n, const unsigned int *nxt, unsigned int *comp,
                                                   unsigned int *best) {
    for (uint64_t v = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; v < n; v += (uint64_t)gridDim.x * blockDim.x) {
        comp[v] = nxt[v];
        best[v] = NONE32;
    }
}

int ec_spanning_forest(const void *cg_edges, uint64_t cg_edge_count, uint64_t cg_vertex_count, uint32_t *tree,
                       uint64_t *tree_count) {
    if (!tree_count || (cg_edge_count && (!cg_edges || !tree))) {
        set_error("null argument");
        return EC_ERR_ARG;
    }
    *tree_count = 0;
    const uint64_t E = cg_edge_count, n = cg_vertex_count;
    if (!E || !n) return EC_OK;
    const CircuitEdge *h = static_cast<const CircuitEdge *>(cg_edges);
    for (uint64_t j = 0; j < E; j++)
        if (h[j].c1 >= n || h[j].c2 >= n) {
            set_error("circuit edge %llu joins circuit %u / %u of %llu", (unsigned long long)j, h[j].c1, h[j].c2,
                      (unsigned long long)n);
            return EC_ERR_ARG;
        }
    EC_DEV(dcg, E * sizeof(CircuitEdge));
    EC_DEV(dcomp, n * 4);
    EC_DEV(dnxt, n * 4);
    EC_DEV(dbest, n * 4);
    EC_DEV(din, E);
    EC_DEV(dany, 4);
    EC_HIP(hipMemcpy(dcg.p, cg_edges, E * sizeof(CircuitEdge), hipMemcpyHostToDevice));
    EC_HIP(hipMemset(din.p, 0, E));
    EC_HIP(hipMemset(dbest.p, 0xFF, n * 4));
    k_iota<<<grid_for(n, 256), 256>>>(dcomp.as<unsigned int>(), n);
    for (int round = 0; round < 64; round++) {  // (<= log2(n) rounds)
        EC_HIP(hipMemset(dany.p, 0, 4));
        k_sf_best<<<grid_for(E, 256), 256>>>(dcg.as<CircuitEdge>(), E, dcomp.as<unsigned int>(),
                                             dbest.as<unsigned int>(), dany.as<unsigned int>());
        unsigned int any = 0;
        EC_HIP(hipMemcpy(&any, dany.p, 4, hipMemcpyDeviceToHost));
        if (!any) break;
        k_sf_hook<<<grid_for(n, 256), 256>>>(dcg.as<CircuitEdge>(), n, dcomp.as<unsigned int>(),
                                             dbest.as<unsigned int>(), dnxt.as<unsigned int>(), din.as<uint8_t>());
        for (int j = 0; j < 64; j++) {  // (<= log2(n) + 1 launches)
            EC_HIP(hipMemset(dany.p, 0, 4));
            k_sf_jump<<<grid_for(n, 256), 256>>>(n, dnxt.as<unsigned int>(), dany.as<unsigned int>());
            EC_HIP(hipMemcpy(&any, dany.p, 4, hipMemcpyDeviceToHost));
            if (!any) break;
        }
        k_sf_settle<<<grid_for(n, 256), 256>>>(n, dnxt.as<unsigned int>(), dcomp.as<unsigned int>(),
                                               dbest.as<unsigned int>());
    }
    std::vector<uint8_t> in(E);
    EC_HIP(hipMemcpy(in.data(), din.p, E, hipMemcpyDeviceToHost));
    uint64_t c = 0;
    for (uint64_t j = 0; j < E; j++)
        if (in[j]) tree[c++] = (uint32_t)j;
    *tree_count = c;
    return EC_OK;
}


// ---- step-level drop-ins (the reference's intermediate module functions) ---------------------
// phase1_device (src/pygpuhash.py:18-73): per-key offset within its bucket + bucket sizes
int ec_hash_phase1(const uint64_t *keys, uint64_t n, uint32_t nb, unsigned flags, uint32_t *offset,
                   uint32_t *bucket_size) {
    if (!nb || (n && (!keys || !offset)) || !bucket_size) {
        set_error("bad arguments");
        return EC_ERR_ARG;
    }
    uint64_t used = n;
    if ((flags & EC_MOD_TAIL_DROP) && n >= 1024) used = (n / 1024) * 1024;
    EC_DEV(dk, used * 8);
    EC_DEV(db, used * 4);
    EC_DEV(di, used * 4);
    EC_DEV(db2, used * 4);
    EC_DEV(di2, used * 4);
    EC_DEV(dsz, nb * 4ull);
    EC_DEV(dst, (nb + 1) * 8ull);
    EC_DEV(doff, used * 4);
    EC_HIP(hipMemset(dsz.p, 0, nb * 4ull));
    if (used) {
        EC_HIP(hipMemcpy(dk.p, keys, used * 8, hipMemcpyHostToDevice));
        k_hash_count<<<grid_for(used, 256), 256>>>(dk.as<unsigned long long>(), used, nb, dsz.as<unsigned int>());
        k_hash_bucket_ids<<<grid_for(used, 256), 256>>>(dk.as<unsigned long long>(), used, nb, db.as<unsigned int>(),
                                                       di.as<unsigned int>());
        size_t bytes = 0;
        EC_HIP(rocprim::radix_sort_pairs(nullptr, bytes, db.as<unsigned int>(), db2.as<unsigned int>(),
                                         di.as<unsigned int>(), di2.as<unsigned int>(), used, 0, 32, (hipStream_t)0));
        EC_DEV(tmp, bytes);
        EC_HIP(rocprim::radix_sort_pairs(tmp.p, bytes, db.as<unsigned int>(), db2.as<unsigned int>(),
                                         di.as<unsigned int>(), di2.as<unsigned int>(), used, 0, 32, (hipStream_t)0));
        EC_CHECK(exscan_u64(dsz.as<unsigned int>(), dst.as<unsigned long long>(), nb));
        k_hash_offsets<<<grid_for(used, 256), 256>>>(di2.as<unsigned int>(), db2.as<unsigned int>(), used,
                                                    dst.as<unsigned long long>(), doff.as<unsigned int>());
        EC_HIP(hipMemcpy(offset, doff.p, used * 4, hipMemcpyDeviceToHost));
    }
    for (uint64_t i = used; i < n; i++) offset[i] = 0;  // never processed by the dropped blocks
    EC_HIP(hipMemcpy(bucket_size, dsz.p, nb * 4ull, hipMemcpyDeviceToHost));
    return EC_OK;
}

// copy_to_bucket_device (src/pygpuhash.py:76-170): bufferK/V[start[b] + offset[i]] = key/value
int ec_hash_copy_to_bucket(const uint64_t *keys, const uint32_t *vals, const uint32_t *offset, uint64_t n,
                           const uint32_t *start, uint32_t nb, uint64_t *buf_k, uint32_t *buf_v, uint64_t buf_len) {
    if (!nb || !start || (n && (!keys || !vals || !offset || !buf_k || !buf_v))) {
        set_error("bad arguments");
        return EC_ERR_ARG;
    }
    std::vector<uint32_t> sz(nb, 0);
    for (uint64_t i = 0; i < n; i++) {
        const uint64_t p = (uint64_t)start[hash_h(keys[i], nb)] + offset[i];
        if (p >= buf_len) {
            set_error("key %llu lands at %llu outside the %llu-entry bucket buffer", (unsigned long long)i,
                      (unsigned long long)p, (unsigned long long)buf_len);
            return EC_ERR_ARG;
        }
    }
    if (!n) return EC_OK;
    EC_DEV(dk, n * 8);
    EC_DEV(dv, n * 4);
    EC_DEV(doff, n * 4);
    EC_DEV(dst, nb * 4ull);
    EC_DEV(dbk, buf_len * 8);
    EC_DEV(dbv, buf_len * 4);
    EC_HIP(hipMemcpy(dk.p, keys, n * 8, hipMemcpyHostToDevice));
    EC_HIP(hipMemcpy(dv.p, vals, n * 4, hipMemcpyHostToDevice));
    EC_HIP(hipMemcpy(doff.p, offset, n * 4, hipMemcpyHostToDevice));
    EC_HIP(hipMemcpy(dst.p, start, nb * 4ull, hipMemcpyHostToDevice));
    EC_HIP(hipMemcpy(dbk.p, buf_k, buf_len * 8, hipMemcpyHostToDevice));
    EC_HIP(hipMemcpy(dbv.p, buf_v, buf_len * 4, hipMemcpyHostToDevice));
    k_hash_copy<<<grid_for(n, 256), 256>>>(dk.as<unsigned long long>(), dv.as<unsigned int>(), doff.as<unsigned int>(), n,
                                          nb, dst.as<unsigned int>(), dbk.as<unsigned long long>(), dbv.as<unsigned int>());
    EC_HIP(hipMemcpy(buf_k, dbk.p, buf_len * 8, hipMemcpyDeviceToHost));
    EC_HIP(hipMemcpy(buf_v, dbv.p, buf_len * 4, hipMemcpyDeviceToHost));
    return EC_OK;
}

// bucket_sort_device (src/pygpuhash.py:173-258): per-bucket rank sort into TK/TV[nb*520]
int ec_hash_bucket_sort(const uint64_t *buf_k, const uint32_t *buf_v, uint64_t buf_len, const uint32_t *start,
                        const uint32_t *bucket_size, uint32_t nb, uint64_t *TK, uint32_t *TV) {
    if (!nb || !start || !bucket_size || !TK || !TV || (buf_len && (!buf_k || !buf_v))) {
        set_error("bad arguments");
        return EC_ERR_ARG;
    }
    for (uint32_t b = 0; b < nb; b++)
        if (bucket_size[b] > BUCKET_ITEMS || (uint64_t)start[b] + bucket_size[b] > buf_len) {
            set_error("bucket %u: size %u / start %u outside the buffer or > 520", b, bucket_size[b], start[b]);
            return EC_ERR_CAPACITY;
        }
    const uint64_t slots = (uint64_t)nb * BUCKET_ITEMS;
    std::vector<unsigned long long> st64(nb);
    for (uint32_t b = 0; b < nb; b++) st64[b] = start[b];
    EC_DEV(dbk, buf_len * 8);
    EC_DEV(dbv, buf_len * 4);
    EC_DEV(didx, buf_len * 4);
    EC_DEV(dst, nb * 8ull);
    EC_DEV(dsz, nb * 4ull);
    EC_DEV(dTK, slots * 8);
    EC_DEV(dTV, slots * 4);
    std::vector<uint32_t> iota(buf_len);
    for (uint64_t i = 0; i < buf_len; i++) iota[i] = (uint32_t)i;
    if (buf_len) {
        EC_HIP(hipMemcpy(dbk.p, buf_k, buf_len * 8, hipMemcpyHostToDevice));
        EC_HIP(hipMemcpy(dbv.p, buf_v, buf_len * 4, hipMemcpyHostToDevice));
        EC_HIP(hipMemcpy(didx.p, iota.data(), buf_len * 4, hipMemcpyHostToDevice));
    }
    EC_HIP(hipMemcpy(dst.p, st64.data(), nb * 8ull, hipMemcpyHostToDevice));
    EC_HIP(hipMemcpy(dsz.p, bucket_size, nb * 4ull, hipMemcpyHostToDevice));
    EC_HIP(hipMemcpy(dTK.p, TK, slots * 8, hipMemcpyHostToDevice));
    EC_HIP(hipMemcpy(dTV.p, TV, slots * 4, hipMemcpyHostToDevice));
    k_hash_bucket_sort<<<nb, 256>>>(dbk.as<unsigned long long>(), didx.as<unsigned int>(), dst.as<unsigned long long>(),
                                    dsz.as<unsigned int>(), dbv.as<unsigned int>(), dTK.as<unsigned long long>(),
                                    dTV.as<unsigned int>());
    EC_HIP(hipMemcpy(TK, dTK.p, slots * 8, hipMemcpyDeviceToHost));
    EC_HIP(hipMemcpy(TV, dTV.p, slots * 4, hipMemcpyDeviceToHost));
    return EC_OK;
}

// assign_successor_device (src/pyeulertour.py:17-107): ee[e[ep+i]].s = l[lp+i]
int ec_assign_successor(const void *ev, uint64_t vcount, const uint32_t *l, const uint32_t *e, void *ee, uint64_t E) {
    if ((vcount && !ev) || (E && (!l || !e || !ee))) {
        set_error("null argument");
        return EC_ERR_ARG;
    }
    if (!E || !vcount) return EC_OK;
    EC_DEV(dev, vcount * sizeof(EulerVertex));
    EC_DEV(dl, E * 4);
    EC_DEV(de, E * 4);
    EC_DEV(dee, E * sizeof(EulerEdge));
    EC_HIP(hipMemcpy(dev.p, ev, vcount * sizeof(EulerVertex), hipMemcpyHostToDevice));
    EC_HIP(hipMemcpy(dl.p, l, E * 4, hipMemcpyHostToDevice));
    EC_HIP(hipMemcpy(de.p, e, E * 4, hipMemcpyHostToDevice));
    EC_HIP(hipMemcpy(dee.p, ee, E * sizeof(EulerEdge), hipMemcpyHostToDevice));
    k_assign_successor<<<grid_for(vcount, 256), 256>>>(dev.as<EulerVertex>(), vcount, dl.as<unsigned int>(),
                                                      de.as<unsigned int>(), dee.as<EulerEdge>(), E);
    EC_HIP(hipMemcpy(ee, dee.p, E * sizeof(EulerEdge), hipMemcpyDeviceToHost));
    return EC_OK;
}

// construct_successor_graphP1/P2_device (src/pyeulertour.py:109-216): Vertex{eid, s, pred}
int ec_successor_graph(const void *ee, uint64_t E, void *vertices) {
    if (E && (!ee || !vertices)) {
        set_error("null argument");
        return EC_ERR_ARG;
    }
    if (!E) return EC_OK;
    EC_DEV(dee, E * sizeof(EulerEdge));
    EC_DEV(dv, E * sizeof(Vtx));
    EC_HIP(hipMemcpy(dee.p, ee, E * sizeof(EulerEdge), hipMemcpyHostToDevice));
    k_succ_graph1<<<grid_for(E, 256), 256>>>(dee.as<EulerEdge>(), E, dv.as<Vtx>());
    k_succ_graph2<<<grid_for(E, 256), 256>>>(dv.as<Vtx>(), E);
    EC_HIP(hipMemcpy(vertices, dv.p, E * sizeof(Vtx), hipMemcpyDeviceToHost));
    return EC_OK;
}


// debruijn_count_device (src/pydebruijn.py:15-178): lcount/ecount[4V]
int ec_db_counts(const uint64_t *lmer_keys, const uint32_t *lmer_values, uint64_t nl, uint32_t l, const uint64_t *TK,
                 const uint32_t *TV, const uint32_t *bucket_size, uint32_t nb, uint64_t size, uint32_t *lcount,
                 uint32_t *ecount) {
    if (l < 2 || l > 32 || !TK || !TV || !bucket_size || !nb || (nl && (!lmer_keys || !lmer_values)) ||
        (size && (!lcount || !ecount))) {
        set_error("bad arguments");
        return EC_ERR_ARG;
    }
    EC_CHECK(check_table(bucket_size, nb));
    const uint64_t slots = (uint64_t)nb * BUCKET_ITEMS;
    EC_DEV(dTK, slots * 8);
    EC_DEV(dTV, slots * 4);
    EC_DEV(dsz, nb * 4ull);
    EC_DEV(dlk, nl * 8);
    EC_DEV(dlv, nl * 4);
    EC_DEV(dlc, size * 4);
    EC_DEV(dec, size * 4);
    EC_HIP(hipMemcpy(dTK.p, TK, slots * 8, hipMemcpyHostToDevice));
    EC_HIP(hipMemcpy(dTV.p, TV, slots * 4, hipMemcpyHostToDevice));
    EC_HIP(hipMemcpy(dsz.p, bucket_size, nb * 4ull, hipMemcpyHostToDevice));
    if (nl) {
        EC_HIP(hipMemcpy(dlk.p, lmer_keys, nl * 8, hipMemcpyHostToDevice));
        EC_HIP(hipMemcpy(dlv.p, lmer_values, nl * 4, hipMemcpyHostToDevice));
    }
    if (size) {
        EC_HIP(hipMemcpy(dlc.p, lcount, size * 4, hipMemcpyHostToDevice));
        EC_HIP(hipMemcpy(dec.p, ecount, size * 4, hipMemcpyHostToDevice));
    }
    const HashView h{dTK.as<unsigned long long>(), dTV.as<unsigned int>(), dsz.as<unsigned int>(), nb};
    if (nl)
        k_db_count<<<grid_for(nl, 256), 256>>>(dlk.as<unsigned long long>(), dlv.as<unsigned int>(), nl, h,
                                              kmask64((int)l - 1), size, dlc.as<unsigned int>(), dec.as<unsigned int>());
    if (size) {
        EC_HIP(hipMemcpy(lcount, dlc.p, size * 4, hipMemcpyDeviceToHost));
        EC_HIP(hipMemcpy(ecount, dec.p, size * 4, hipMemcpyDeviceToHost));
    }
    return EC_OK;
}

// setup_vertices_device (src/pydebruijn.py:181-324)
int ec_db_vertices(const uint64_t *kmer_keys, uint64_t nk, const uint64_t *TK, const uint32_t *TV,
                   const uint32_t *bucket_size, uint32_t nb, const uint32_t *lcount, const uint32_t *lstart,
                   const uint32_t *ecount, const uint32_t *estart, void *ev) {
    if (!TK || !TV || !bucket_size || !nb || (nk && (!kmer_keys || !lcount || !lstart || !ecount || !estart || !ev))) {
        set_error("bad arguments");
        return EC_ERR_ARG;
    }
    EC_CHECK(check_table(bucket_size, nb));
    if (!nk) return EC_OK;
    const uint64_t slots = (uint64_t)nb * BUCKET_ITEMS, size = 4 * nk;
    EC_DEV(dTK, slots * 8);
    EC_DEV(dTV, slots * 4);
    EC_DEV(dsz, nb * 4ull);
    EC_DEV(dkk, nk * 8);
    EC_DEV(dlc, size * 4);
    EC_DEV(dls, size * 4);
    EC_DEV(dec, size * 4);
    EC_DEV(des, size * 4);
    EC_DEV(dev, nk * sizeof(EulerVertex));
    EC_HIP(hipMemcpy(dTK.p, TK, slots * 8, hipMemcpyHostToDevice));
    EC_HIP(hipMemcpy(dTV.p, TV, slots * 4, hipMemcpyHostToDevice));
    EC_HIP(hipMemcpy(dsz.p, bucket_size, nb * 4ull, hipMemcpyHostToDevice));
    EC_HIP(hipMemcpy(dkk.p, kmer_keys, nk * 8, hipMemcpyHostToDevice));
    EC_HIP(hipMemcpy(dlc.p, lcount, size * 4, hipMemcpyHostToDevice));
    EC_HIP(hipMemcpy(dls.p, lstart, size * 4, hipMemcpyHostToDevice));
    EC_HIP(hipMemcpy(dec.p, ecount, size * 4, hipMemcpyHostToDevice));
    EC_HIP(hipMemcpy(des.p, estart, size * 4, hipMemcpyHostToDevice));
    EC_HIP(hipMemcpy(dev.p, ev, nk * sizeof(EulerVertex), hipMemcpyHostToDevice));
    const HashView h{dTK.as<unsigned long long>(), dTV.as<unsigned int>(), dsz.as<unsigned int>(), nb};
    k_db_vertices<<<grid_for(nk, 256), 256>>>(dkk.as<unsigned long long>(), nk, h, dlc.as<unsigned int>(),
                                             dls.as<unsigned int>(), dec.as<unsigned int>(), des.as<unsigned int>(),
                                             dev.as<EulerVertex>());
    EC_HIP(hipMemcpy(ev, dev.p, nk * sizeof(EulerVertex), hipMemcpyDeviceToHost));
    return EC_OK;
}

// setup_edges_device (src/pydebruijn.py:326-512); E = length of ee / l / e
int ec_db_edges(const uint64_t *lmer_keys, const uint32_t *lmer_values, const uint32_t *lmer_offsets, uint64_t nl,
                uint32_t l, const uint64_t *TK, const uint32_t *TV, const uint32_t *bucket_size, uint32_t nb,
                uint64_t nk, const uint32_t *lstart, const uint32_t *estart, unsigned flags, void *ee, uint32_t *l_out,
                uint32_t *e_out, uint64_t E) {
    if (l < 2 || l > 32 || !TK || !TV || !bucket_size || !nb || (nl && (!lmer_keys || !lmer_values || !lmer_offsets)) ||
        (nk && (!lstart || !estart)) || (E && (!ee || !l_out || !e_out))) {
        set_error("bad arguments");
        return EC_ERR_ARG;
    }
    EC_CHECK(check_table(bucket_size, nb));
    const uint64_t slots = (uint64_t)nb * BUCKET_ITEMS, size = 4 * nk;
    EC_DEV(dTK, slots * 8);
    EC_DEV(dTV, slots * 4);
    EC_DEV(dsz, nb * 4ull);
    EC_DEV(dlk, nl * 8);
    EC_DEV(dlv, nl * 4);
    EC_DEV(dlo, nl * 4);
    EC_DEV(dls, size * 4);
    EC_DEV(des, size * 4);
    EC_DEV(dee, E * sizeof(EulerEdge));
    EC_DEV(dl, E * 4);
    EC_DEV(de, E * 4);
    EC_HIP(hipMemcpy(dTK.p, TK, slots * 8, hipMemcpyHostToDevice));
    EC_HIP(hipMemcpy(dTV.p, TV, slots * 4, hipMemcpyHostToDevice));
    EC_HIP(hipMemcpy(dsz.p, bucket_size, nb * 4ull, hipMemcpyHostToDevice));
    if (nl) {
        EC_HIP(hipMemcpy(dlk.p, lmer_keys, nl * 8, hipMemcpyHostToDevice));
        EC_HIP(hipMemcpy(dlv.p, lmer_values, nl * 4, hipMemcpyHostToDevice));
        EC_HIP(hipMemcpy(dlo.p, lmer_offsets, nl * 4, hipMemcpyHostToDevice));
    }
    if (size) {
        EC_HIP(hipMemcpy(dls.p, lstart, size * 4, hipMemcpyHostToDevice));
        EC_HIP(hipMemcpy(des.p, estart, size * 4, hipMemcpyHostToDevice));
    }
    if (E) {
        EC_HIP(hipMemcpy(dee.p, ee, E * sizeof(EulerEdge), hipMemcpyHostToDevice));
        EC_HIP(hipMemcpy(dl.p, l_out, E * 4, hipMemcpyHostToDevice));
        EC_HIP(hipMemcpy(de.p, e_out, E * 4, hipMemcpyHostToDevice));
    }
    const HashView h{dTK.as<unsigned long long>(), dTV.as<unsigned int>(), dsz.as<unsigned int>(), nb};
    if (nl)
        k_db_edges<<<grid_for(nl, 256), 256>>>(dlk.as<unsigned long long>(), dlv.as<unsigned int>(),
                                              dlo.as<unsigned int>(), nl, h, kmask64((int)l - 1), size, E,
                                              (flags & EC_MOD_REF_BOUNDS) ? 1 : 0, dls.as<unsigned int>(),
                                              des.as<unsigned int>(), dl.as<unsigned int>(), de.as<unsigned int>(),
                                              dee.as<EulerEdge>());
    if (E) {
        EC_HIP(hipMemcpy(ee, dee.p, E * sizeof(EulerEdge), hipMemcpyDeviceToHost));
        EC_HIP(hipMemcpy(l_out, dl.p, E * 4, hipMemcpyDeviceToHost));
        EC_HIP(hipMemcpy(e_out, de.p, E * 4, hipMemcpyDeviceToHost));
    }
    return EC_OK;
}

}  // extern "C"


// readLmersKmersCuda (src/eulercuda.py:73-179) on the device: encode F / RC l-mers of the
// concatenated buffer, split them, and dedup both streams in first-occurrence order.
// Capacities: lmer_keys / lmer_values 2B, kmer_keys 4B.
static int unique_first(const unsigned long long *keys, uint64_t n, int skip_zero, unsigned long long *out_k,
                        unsigned int *out_c, uint64_t *nu_out) {
    *nu_out = 0;
    if (!n) return EC_OK;
    EC_DEV(idx, n * 4);
    EC_DEV(sk, n * 8);
    EC_DEV(si, n * 4);
    EC_DEV(flag, n * 4);
    EC_DEV(pos, n * 4);
    k_iota<<<grid_for(n, 256), 256>>>(idx.as<unsigned int>(), n);
    size_t bytes = 0;
    EC_HIP(rocprim::radix_sort_pairs(nullptr, bytes, keys, sk.as<unsigned long long>(), idx.as<unsigned int>(),
                                     si.as<unsigned int>(), n, 0, 64, (hipStream_t)0));
    {
        EC_DEV(tmp, bytes);
        EC_HIP(rocprim::radix_sort_pairs(tmp.p, bytes, keys, sk.as<unsigned long long>(), idx.as<unsigned int>(),
                                         si.as<unsigned int>(), n, 0, 64, (hipStream_t)0));
    }
    k_seg_heads<<<grid_for(n, 256), 256>>>(sk.as<unsigned long long>(), n, skip_zero, flag.as<unsigned int>());
    EC_CHECK(exscan_u32(flag.as<unsigned int>(), pos.as<unsigned int>(), n));
    uint32_t last[2];
    EC_HIP(hipMemcpy(&last[0], pos.as<unsigned int>() + (n - 1), 4, hipMemcpyDeviceToHost));
    EC_HIP(hipMemcpy(&last[1], flag.as<unsigned int>() + (n - 1), 4, hipMemcpyDeviceToHost));
    const uint64_t nu = (uint64_t)last[0] + last[1];
    *nu_out = nu;
    if (!nu) return EC_OK;
    EC_DEV(uk, nu * 8);
    EC_DEV(ufirst, nu * 4);
    EC_DEV(ustart, nu * 4);
    EC_DEV(sfirst, nu * 4);
    EC_DEV(ord0, nu * 4);
    EC_DEV(ord, nu * 4);
    k_seg_compact<<<grid_for(n, 256), 256>>>(sk.as<unsigned long long>(), si.as<unsigned int>(), flag.as<unsigned int>(),
                                             pos.as<unsigned int>(), n, uk.as<unsigned long long>(),
                                             ufirst.as<unsigned int>(), ustart.as<unsigned int>());
    k_iota<<<grid_for(nu, 256), 256>>>(ord0.as<unsigned int>(), nu);
    bytes = 0;
    EC_HIP(rocprim::radix_sort_pairs(nullptr, bytes, ufirst.as<unsigned int>(), sfirst.as<unsigned int>(),
                                     ord0.as<unsigned int>(), ord.as<unsigned int>(), nu, 0, 32, (hipStream_t)0));
    {
        EC_DEV(tmp, bytes);
        EC_HIP(rocprim::radix_sort_pairs(tmp.p, bytes, ufirst.as<unsigned int>(), sfirst.as<unsigned int>(),
                                         ord0.as<unsigned int>(), ord.as<unsigned int>(), nu, 0, 32, (hipStream_t)0));
    }
    k_seg_emit<<<grid_for(nu, 256), 256>>>(ord.as<unsigned int>(), uk.as<unsigned long long>(), ustart.as<unsigned int>(),
                                           nu, n, out_k, out_c);
    return EC_OK;
}

extern "C" int ec_read_lmers_kmers(const uint8_t *buf, uint64_t B, uint32_t L, uint64_t *lmer_keys,
                                   uint32_t *lmer_values, uint64_t *n_lmers, uint64_t *lmer_empty, uint64_t *kmer_keys,
                                   uint64_t *n_kmers) {
    if (L < 2 || L > 32 || !n_lmers || !lmer_empty || !n_kmers || (B && (!buf || !lmer_keys || !lmer_values || !kmer_keys))) {
        set_error("bad arguments (L=%u must be in [2,32])", L);
        return EC_ERR_ARG;
    }
    *n_lmers = *lmer_empty = *n_kmers = 0;
    if (!B) return EC_OK;
    if (4 * B >= (1ull << 32)) {
        set_error("buffer of %llu bases exceeds the 2^30 limit of the module path", (unsigned long long)B);
        return EC_ERR_CAPACITY;
    }
    EC_DEV(db, B);
    EC_DEV(F, B * 8);
    EC_DEV(R, B * 8);
    EC_DEV(S, 2 * B * 8);
    EC_DEV(K, 4 * B * 8);
    EC_DEV(zc, 8);
    EC_DEV(ok, 2 * B * 8);
    EC_DEV(oc, 2 * B * 4);
    EC_DEV(okk, 4 * B * 8);
    EC_HIP(hipMemcpy(db.p, buf, B, hipMemcpyHostToDevice));
    k_encode_lmer<<<grid_for(B, 256, 65535), 256>>>(db.as<uint8_t>(), B, L, 0, F.as<unsigned long long>());
    k_encode_lmer<<<grid_for(B, 256, 65535), 256>>>(db.as<uint8_t>(), B, L, 1, R.as<unsigned long long>());
    k_streams<<<grid_for(B, 256), 256>>>(F.as<unsigned long long>(), R.as<unsigned long long>(), B, kmask64((int)L - 1),
                                         S.as<unsigned long long>(), K.as<unsigned long long>());
    EC_HIP(hipMemset(zc.p, 0, 8));
    k_count_zero<<<grid_for(2 * B, 256, 4096), 256>>>(S.as<unsigned long long>(), 2 * B, zc.as<unsigned long long>());
    uint64_t nl = 0, nk = 0, empty = 0;
    EC_CHECK(unique_first(S.as<unsigned long long>(), 2 * B, 1, ok.as<unsigned long long>(), oc.as<unsigned int>(), &nl));
    EC_CHECK(unique_first(K.as<unsigned long long>(), 4 * B, 0, okk.as<unsigned long long>(), nullptr, &nk));
    EC_HIP(hipMemcpy(&empty, zc.p, 8, hipMemcpyDeviceToHost));
    if (nl) {
        EC_HIP(hipMemcpy(lmer_keys, ok.p, nl * 8, hipMemcpyDeviceToHost));
        EC_HIP(hipMemcpy(lmer_values, oc.p, nl * 4, hipMemcpyDeviceToHost));
    }
    if (nk) EC_HIP(hipMemcpy(kmer_keys, okk.p, nk * 8, hipMemcpyDeviceToHost));
    *n_lmers = nl;
    *n_kmers = nk;
    *lmer_empty = empty;
    return EC_OK;
}

// generatePartialContig (src/eulercuda.py:328-402) on the device for an injective successor
// map: contig c = chars[coff[c] .. coff[c+1]), the getString(l-1, vid) of every walked edge's
// source vertex followed by the last edge's target vertex.  chars capacity: 2E(l-1);
// coff capacity E+1.
extern "C" int ec_partial_contigs(const void *ev, uint64_t vcount, const void *ee, uint64_t E, uint32_t l, char *chars,
                                  uint64_t *coff, uint64_t *n_contigs, uint64_t *n_chars) {
    if (l < 2 || l > 33 || !n_contigs || !n_chars || (E && (!ee || !chars || !coff || !ev))) {
        set_error("bad arguments (l=%u must be in [2,33])", l);
        return EC_ERR_ARG;
    }
    *n_contigs = *n_chars = 0;
    if (!E) {
        if (coff) coff[0] = 0;
        return EC_OK;
    }
    if (E >= (1ull << 31)) {
        set_error("%llu edges exceed the 2^31 limit", (unsigned long long)E);
        return EC_ERR_CAPACITY;
    }
    const unsigned int km1 = l - 1;
    EC_DEV(dev, vcount * sizeof(EulerVertex));
    EC_DEV(dee, E * sizeof(EulerEdge));
    EC_DEV(pred, E * 4);
    EC_DEV(indeg, E * 4);
    EC_DEV(nxt, E * 4);
    EC_DEV(d, E * 4);
    EC_DEV(hd, E * 4);
    EC_DEV(mn, E * 4);
    EC_DEV(nxt2, E * 4);
    EC_DEV(d2, E * 4);
    EC_DEV(hd2, E * 4);
    EC_DEV(mn2, E * 4);
    EC_DEV(cmin, E * 4);
    EC_DEV(key, E * 8);
    EC_DEV(val, E * 4);
    EC_DEV(skey, E * 8);
    EC_DEV(sval, E * 4);
    EC_DEV(len, E * 8);
    EC_DEV(pos, E * 8);
    EC_DEV(start, E * 4);
    EC_DEV(cidx, E * 4);
    EC_DEV(bad, 4);
    if (vcount) EC_HIP(hipMemcpy(dev.p, ev, vcount * sizeof(EulerVertex), hipMemcpyHostToDevice));
    EC_HIP(hipMemcpy(dee.p, ee, E * sizeof(EulerEdge), hipMemcpyHostToDevice));
    EC_HIP(hipMemset(pred.p, 0xFF, E * 4));
    EC_HIP(hipMemset(indeg.p, 0, E * 4));
    EC_HIP(hipMemset(bad.p, 0, 4));
    k_pw_pred<<<grid_for(E, 256), 256>>>(dee.as<EulerEdge>(), E, pred.as<unsigned int>(), indeg.as<unsigned int>());
    {
        size_t bytes = 0;
        EC_DEV(mx, 4);
        EC_HIP(rocprim::reduce(nullptr, bytes, indeg.as<unsigned int>(), mx.as<unsigned int>(), 0u, E,
                               rocprim::maximum<unsigned int>(), (hipStream_t)0));
        EC_DEV(tmp, bytes);
        EC_HIP(rocprim::reduce(tmp.p, bytes, indeg.as<unsigned int>(), mx.as<unsigned int>(), 0u, E,
                               rocprim::maximum<unsigned int>(), (hipStream_t)0));
        unsigned int h = 0;
        EC_HIP(hipMemcpy(&h, mx.p, 4, hipMemcpyDeviceToHost));
        if (h > 1) {
            set_error("successor map is not injective (an edge is the successor of %u edges)", h);
            return EC_ERR_ARG;
        }
    }
    int rounds = 1;
    while ((1ull << rounds) <= E) rounds++;
    rounds++;
    const unsigned int *cut = nullptr;
    for (int pass = 0; pass < 2; pass++) {
        k_pw_init<<<grid_for(E, 256), 256>>>(pred.as<unsigned int>(), cut, E, nxt.as<unsigned int>(), d.as<unsigned int>(),
                                             hd.as<unsigned int>(), mn.as<unsigned int>());
        unsigned int *a[4] = {nxt.as<unsigned int>(), d.as<unsigned int>(), hd.as<unsigned int>(), mn.as<unsigned int>()};
        unsigned int *b[4] = {nxt2.as<unsigned int>(), d2.as<unsigned int>(), hd2.as<unsigned int>(), mn2.as<unsigned int>()};
        for (int r = 0; r < rounds; r++) {
            k_pw_jump<<<grid_for(E, 256), 256>>>(a[0], a[1], a[2], a[3], E, b[0], b[1], b[2], b[3]);
            for (int q = 0; q < 4; q++) std::swap(a[q], b[q]);
        }
        if (pass == 0) {
            k_pw_cycmin<<<grid_for(E, 256), 256>>>(a[0], a[3], E, cmin.as<unsigned int>());
            cut = cmin.as<unsigned int>();
        } else {
            k_pw_keys<<<grid_for(E, 256), 256>>>(cmin.as<unsigned int>(), a[2], a[1], E, key.as<unsigned long long>(),
                                                 val.as<unsigned int>());
        }
    }
    {
        size_t bytes = 0;
        EC_HIP(rocprim::radix_sort_pairs(nullptr, bytes, key.as<unsigned long long>(), skey.as<unsigned long long>(),
                                         val.as<unsigned int>(), sval.as<unsigned int>(), E, 0, 64, (hipStream_t)0));
        EC_DEV(tmp, bytes);
        EC_HIP(rocprim::radix_sort_pairs(tmp.p, bytes, key.as<unsigned long long>(), skey.as<unsigned long long>(),
                                         val.as<unsigned int>(), sval.as<unsigned int>(), E, 0, 64, (hipStream_t)0));
    }
    k_pw_len<<<grid_for(E, 256), 256>>>(skey.as<unsigned long long>(), E, km1, len.as<unsigned long long>(),
                                        start.as<unsigned int>());
    {
        size_t bytes = 0;
        EC_HIP(rocprim::exclusive_scan(nullptr, bytes, len.as<unsigned long long>(), pos.as<unsigned long long>(), 0ull, E,
                                       rocprim::plus<unsigned long long>(), (hipStream_t)0));
        EC_DEV(tmp, bytes);
        EC_HIP(rocprim::exclusive_scan(tmp.p, bytes, len.as<unsigned long long>(), pos.as<unsigned long long>(), 0ull, E,
                                       rocprim::plus<unsigned long long>(), (hipStream_t)0));
        bytes = 0;
        EC_HIP(rocprim::inclusive_scan(nullptr, bytes, start.as<unsigned int>(), cidx.as<unsigned int>(), E,
                                       rocprim::plus<unsigned int>(), (hipStream_t)0));
        EC_DEV(tmp2, bytes);
        EC_HIP(rocprim::inclusive_scan(tmp2.p, bytes, start.as<unsigned int>(), cidx.as<unsigned int>(), E,
                                       rocprim::plus<unsigned int>(), (hipStream_t)0));
    }
    unsigned long long lastpos = 0, lastlen = 0;
    unsigned int nc = 0;
    EC_HIP(hipMemcpy(&lastpos, pos.as<unsigned long long>() + (E - 1), 8, hipMemcpyDeviceToHost));
    EC_HIP(hipMemcpy(&lastlen, len.as<unsigned long long>() + (E - 1), 8, hipMemcpyDeviceToHost));
    EC_HIP(hipMemcpy(&nc, cidx.as<unsigned int>() + (E - 1), 4, hipMemcpyDeviceToHost));
    const uint64_t total = lastpos + lastlen;
    EC_DEV(dchars, total);
    EC_DEV(dcoff, (nc + 1ull) * 8);
    k_pw_emit<<<grid_for(E, 256), 256>>>(skey.as<unsigned long long>(), sval.as<unsigned int>(),
                                         pos.as<unsigned long long>(), cidx.as<unsigned int>(), E, dee.as<EulerEdge>(),
                                         dev.as<EulerVertex>(), vcount, km1, dchars.as<char>(),
                                         dcoff.as<unsigned long long>(), bad.as<unsigned int>());
    unsigned int hb = 0;
    EC_HIP(hipMemcpy(&hb, bad.p, 4, hipMemcpyDeviceToHost));
    if (hb) {
        set_error("an edge names a vertex outside ev[0..%llu)", (unsigned long long)vcount);
        return EC_ERR_ARG;
    }
    EC_HIP(hipMemcpy(chars, dchars.p, total, hipMemcpyDeviceToHost));
    EC_HIP(hipMemcpy(coff, dcoff.p, nc * 8ull, hipMemcpyDeviceToHost));
    coff[nc] = total;
    *n_contigs = nc;
    *n_chars = total;
    return EC_OK;
}

// ---- Shiloach-Vishkin steps of find_component_device, one launch each (round 5) ---------------
// src/pycomponent.py:16-665: the ten step kernels the reference's component loop is made of,
// exposed step by step (ec_component_step) with the reference's arguments and in-place
// semantics.  Every step is elementwise over tid < length; the atomics of steps 2/3 (P2) are
// minima and same-value stores, so the result does not depend on thread order.  Indices the
// reference would read out of bounds (a D / prevD / val entry >= length) are skipped.
namespace ec {
enum SvStep : int {
    SV_INIT = 0,      // componentStepInit (:34-43): D = tid, Q = 0
    SV_S1P1 = 1,      // componentStepOne_ShortCuttingP1 (:87-94): D = prevD[prevD]
    SV_S1P2 = 2,      // componentStepOne_ShortCuttingP2 (:148-158): D != prevD -> Q[D] = s
    SV_S2P1 = 3,      // componentStepTwoP1 (:212-242): hook candidates of unchanged roots
    SV_S2P2 = 4,      // componentStepTwoP2 (:301-330): atomicMin(D + t, val), Q[val] = s
    SV_S3P1 = 5,      // componentStepThreeP1 (:394-414): hook candidates of stagnant stars
    SV_S3P2 = 6,      // componentStepThreeP2 (:474-494): atomicMin(D + t, val)
    SV_S4P1 = 7,      // componentStepFourP1 (:548-553): val1 = D[D]
    SV_S4P2 = 8,      // componentStepFourP2 (:595-601): D = val1
    SV_S5 = 9,        // componentStepFive (:638-646): any Q == s -> *sptemp = 1
};

__global__ void __launch_bounds__(256) k_sv_step(int step, const Vtx *v, const unsigned int *prevD, unsigned int *D,
                                                 unsigned int *Q, unsigned int *t1, unsigned int *val1,
                                                 unsigned int *t2, unsigned int *val2, unsigned int *sptemp,
                                                 unsigned int n, unsigned int s) {
    for (unsigned int t = blockIdx.x * blockDim.x + threadIdx.x; t < n; t += gridDim.x * blockDim.x) {
        switch (step) {
        case SV_INIT:
            D[t] = t;
            Q[t] = 0;
            break;
        case SV_S1P1: {
            const unsigned int p = prevD[t];
            if (p < n) D[t] = prevD[p];
            break;
        }
        case SV_S1P2:
            if (D[t] != prevD[t] && D[t] < n) Q[D[t]] = s;
            break;
        case SV_S2P1:
        case SV_S3P1: {
            const unsigned int d = D[t];
            t1[t] = n;
            t2[t] = n;
            bool live;
            if (step == SV_S2P1) live = d == prevD[t];
            else live = d < n && d == D[d] && Q[d] < s;
            if (!live) break;
            const unsigned int nb[2] = {v[t].n1, v[t].n2};
            for (int q = 0; q < 2; q++) {
                if (nb[q] >= n) continue;
                const unsigned int dn = D[nb[q]];
                if (step == SV_S2P1 ? dn < d : dn != d) {
                    (q ? t2 : t1)[t] = d;
                    (q ? val2 : val1)[t] = dn;
                }
            }
            break;
        }
        case SV_S2P2:
        case SV_S3P2:
            for (int q = 0; q < 2; q++) {
                const unsigned int a = (q ? t2 : t1)[t], val = (q ? val2 : val1)[t];
                if (a >= n) continue;
                atomicMin(D + a, val);
                if (step == SV_S2P2 && val < n) Q[val] = s;  // (atomicExch of one value s)
            }
            break;
        case SV_S4P1: {
            const unsigned int d = D[t];
            if (d < n) val1[t] = D[d];
            break;
        }
        case SV_S4P2:
            D[t] = val1[t];
            break;
        case SV_S5:
            if (Q[t] == s) *sptemp = 1;  // (atomicExch of one value)
            break;
        }
    }
}

// calculateCircuitGraphVertexData (src/pyeulertour.py:223-231): C[D[tid]] = 1
__global__ void __launch_bounds__(256) k_circuit_mark_checked(const unsigned int *D, uint64_t n, unsigned int *C,
                                                              uint64_t nc, unsigned int *bad) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < n; t += (uint64_t)gridDim.x * blockDim.x) {
        if (D[t] < nc) C[D[t]] = 1;
        else atomicOr(bad, 1u);
    }
}
// constructCircuitGraphVertex (:280-288): cv[offset[tid]] = tid where C[tid] != 0
__global__ void __launch_bounds__(256) k_cg_vertex(const unsigned int *C, const unsigned int *offset, unsigned int n,
                                                   unsigned int *cv, unsigned int ncv) {
    for (unsigned int t = blockIdx.x * blockDim.x + threadIdx.x; t < n; t += gridDim.x * blockDim.x)
        if (C[t] != 0 && offset[t] < ncv) cv[offset[t]] = t;
}

// calculateCircuitGraphEdgeData (:331-371) / assignCircuitGraphEdgeData (:428-469), per vertex:
// the candidate circuit-graph edges (consecutive entering edges on different circuits) in
// the order a sequential run of the kernel's threads meets them (vertex, then entry index)
__device__ inline bool cg_pair(const unsigned int *e, const unsigned int *D, const unsigned int *map, unsigned int E,
                               unsigned int nmap, unsigned int index, unsigned int &c1, unsigned int &c2) {
    if (index + 1 >= E || e[index] >= E || e[index + 1] >= E) return false;
    const unsigned int d1 = D[e[index]], d2 = D[e[index + 1]];
    if (d1 >= nmap || d2 >= nmap) return false;
    c1 = map[d1];
    c2 = map[d2];
    return c1 != c2;
}
__global__ void __launch_bounds__(256) k_cg_count(const EulerVertex *ev, unsigned int vcount, const unsigned int *e,
                                                  const unsigned int *D, const unsigned int *map, unsigned int E,
                                                  unsigned int nmap, unsigned int *per_vertex,
                                                  unsigned int *cedge_count, unsigned int ngroups, unsigned int *bad) {
    for (unsigned int t = blockIdx.x * blockDim.x + threadIdx.x; t < vcount; t += gridDim.x * blockDim.x) {
        const EulerVertex v = ev[t];
        unsigned int c = 0;
        if (v.ecount > 0) {
            const unsigned int maxIndex = v.ep + v.ecount - 1;
            for (unsigned int index = v.ep; index < maxIndex && index < E; index++) {
                unsigned int c1, c2;
                if (!cg_pair(e, D, map, E, nmap, index, c1, c2)) continue;
                c++;
                if (cedge_count) {  // (atomicInc(.., ecount): the count stays below its bound)
                    if (min(c1, c2) < ngroups) atomicAdd(cedge_count + min(c1, c2), 1u);
                    else atomicOr(bad, 1u);
                }
            }
        }
        if (per_vertex) per_vertex[t] = c;
    }
}
// the candidates of vertex t at slots base[t] .. (exclusive scan of k_cg_count's per-vertex
// counts): key = the group c = min(c1, c2), value = the candidate's sequential position
__global__ void __launch_bounds__(256) k_cg_list(const EulerVertex *ev, unsigned int vcount, const unsigned int *e,
                                                 const unsigned int *D, const unsigned int *map, unsigned int E,
                                                 unsigned int nmap, const unsigned int *base, unsigned int *gkey,
                                                 unsigned int *gpos, uint4 *cand) {
    for (unsigned int t = blockIdx.x * blockDim.x + threadIdx.x; t < vcount; t += gridDim.x * blockDim.x) {
        const EulerVertex v = ev[t];
        unsigned int o = base[t];
        if (v.ecount == 0) continue;
        const unsigned int maxIndex = v.ep + v.ecount - 1;
        for (unsigned int index = v.ep; index < maxIndex && index < E; index++) {
            unsigned int c1, c2;
            if (!cg_pair(e, D, map, E, nmap, index, c1, c2)) continue;
            gkey[o] = min(c1, c2);
            gpos[o] = o;
            cand[o] = make_uint4(e[index], e[index + 1], min(c1, c2), max(c1, c2));
            o++;
        }
    }
}
// group-sorted candidates (stable: sequential order inside a group); the r-th candidate of
// group c takes atomicDec's r-th return, i = count[c] - 1 - r, at cedge[offset[c] + i]
__global__ void __launch_bounds__(256) k_cg_assign(const unsigned int *skey, const unsigned int *spos, unsigned int nc,
                                                   const uint4 *cand, const unsigned int *cedge_offset,
                                                   const unsigned int *cedge_count, unsigned int ngroups,
                                                   CircuitEdge *cedge, unsigned int cecount) {
    for (unsigned int j = blockIdx.x * blockDim.x + threadIdx.x; j < nc; j += gridDim.x * blockDim.x) {
        const unsigned int c = skey[j];
        if (c >= ngroups) continue;
        unsigned int lo = 0, hi = j;  // first position of group c (binary search)
        while (lo < hi) {
            const unsigned int mid = (lo + hi) / 2;
            if (skey[mid] < c) lo = mid + 1;
            else hi = mid;
        }
        const unsigned int r = j - lo;
        if (r >= cedge_count[c]) continue;  // (the reference's atomicDec would wrap)
        const unsigned int slot = cedge_offset[c] + cedge_count[c] - 1 - r;
        if (slot >= cecount) continue;
        const uint4 x = cand[spos[j]];
        CircuitEdge &o = cedge[slot];
        o.c1 = x.z;
        o.c2 = x.w;
        o.e1 = x.x;
        o.e2 = x.y;  // (ceid is left as the caller set it, as the reference kernel does)
    }
}
}  // namespace ec

extern "C" {

int ec_component_step(int step, const void *vertices, uint32_t *prevD, uint32_t *D, uint32_t *Q, uint32_t *t1,
                      uint32_t *val1, uint32_t *t2, uint32_t *val2, uint32_t *sptemp, uint64_t length, uint32_t s) {
    if (step < SV_INIT || step > SV_S5 || length >= 0xFFFFFFFFull) {
        set_error("bad component step %d / length %llu", step, (unsigned long long)length);
        return EC_ERR_ARG;
    }
    const uint64_t n = length;
    // which arrays the step reads (r) / writes (w)
    const bool need_v = step == SV_S2P1 || step == SV_S3P1;
    const bool need_prev = step == SV_S1P1 || step == SV_S1P2 || step == SV_S2P1;
    const bool need_D = step != SV_S5;
    const bool need_Q = step == SV_INIT || step == SV_S1P2 || step == SV_S2P2 || step == SV_S3P1 || step == SV_S5;
    const bool need_t = step == SV_S2P1 || step == SV_S2P2 || step == SV_S3P1 || step == SV_S3P2;
    const bool need_val1 = need_t || step == SV_S4P1 || step == SV_S4P2;
    const bool need_s5 = step == SV_S5;
    if (n && ((need_v && !vertices) || (need_prev && !prevD) || (need_D && !D) || (need_Q && !Q) ||
              (need_t && (!t1 || !t2 || !val2)) || (need_val1 && !val1) || (need_s5 && !sptemp))) {
        set_error("component step %d: a required array is null", step);
        return EC_ERR_ARG;
    }
    if (!n) return EC_OK;
    EC_DEV(dv, need_v ? n * sizeof(Vtx) : 16);
    EC_DEV(dprev, need_prev ? n * 4 : 16);
    EC_DEV(dD, n * 4);
    EC_DEV(dQ, n * 4);
    EC_DEV(dt, need_t ? n * 16 : 16);  // t1, val1, t2, val2
    EC_DEV(dval1, n * 4);
    EC_DEV(dsp, 4);
    unsigned int *dt1 = dt.as<unsigned int>(), *dt2 = dt1 + (need_t ? n : 0), *dval2 = dt2 + (need_t ? n : 0);
    if (need_v) EC_HIP(hipMemcpy(dv.p, vertices, n * sizeof(Vtx), hipMemcpyHostToDevice));
    if (need_prev) EC_HIP(hipMemcpy(dprev.p, prevD, n * 4, hipMemcpyHostToDevice));
    if (need_D && step != SV_INIT) EC_HIP(hipMemcpy(dD.p, D, n * 4, hipMemcpyHostToDevice));
    if (need_Q && step != SV_INIT) EC_HIP(hipMemcpy(dQ.p, Q, n * 4, hipMemcpyHostToDevice));
    if (need_t) {  // (P1 leaves val1 / val2 alone where no candidate: their inputs stay)
        EC_HIP(hipMemcpy(dt1, t1, n * 4, hipMemcpyHostToDevice));
        EC_HIP(hipMemcpy(dt2, t2, n * 4, hipMemcpyHostToDevice));
        EC_HIP(hipMemcpy(dval2, val2, n * 4, hipMemcpyHostToDevice));
    }
    if (need_val1) EC_HIP(hipMemcpy(dval1.p, val1, n * 4, hipMemcpyHostToDevice));
    if (need_s5) EC_HIP(hipMemcpy(dsp.p, sptemp, 4, hipMemcpyHostToDevice));
    k_sv_step<<<grid_for(n, 256), 256>>>(step, dv.as<Vtx>(), dprev.as<unsigned int>(), dD.as<unsigned int>(),
                                        dQ.as<unsigned int>(), dt1, dval1.as<unsigned int>(), dt2, dval2,
                                        dsp.as<unsigned int>(), (unsigned int)n, s);
    EC_HIP(hipGetLastError());
    if (need_D) EC_HIP(hipMemcpy(D, dD.p, n * 4, hipMemcpyDeviceToHost));
    if (need_Q) EC_HIP(hipMemcpy(Q, dQ.p, n * 4, hipMemcpyDeviceToHost));
    if (need_t) {
        EC_HIP(hipMemcpy(t1, dt1, n * 4, hipMemcpyDeviceToHost));
        EC_HIP(hipMemcpy(t2, dt2, n * 4, hipMemcpyDeviceToHost));
        EC_HIP(hipMemcpy(val2, dval2, n * 4, hipMemcpyDeviceToHost));
    }
    if (need_val1) EC_HIP(hipMemcpy(val1, dval1.p, n * 4, hipMemcpyDeviceToHost));
    if (need_s5) EC_HIP(hipMemcpy(sptemp, dsp.p, 4, hipMemcpyDeviceToHost));
    return EC_OK;
}

int ec_cg_vertex_data(const uint32_t *D, uint64_t length, uint32_t *C, uint64_t ncount) {
    if (length && (!D || !C)) {
        set_error("null argument");
        return EC_ERR_ARG;
    }
    if (!length) return EC_OK;
    EC_DEV(dD, length * 4);
    EC_DEV(dC, ncount * 4);
    EC_HIP(hipMemcpy(dD.p, D, length * 4, hipMemcpyHostToDevice));
    EC_HIP(hipMemcpy(dC.p, C, ncount * 4, hipMemcpyHostToDevice));
    EC_DEV(dbad, 4);
    EC_HIP(hipMemset(dbad.p, 0, 4));
    k_circuit_mark_checked<<<grid_for(length, 256), 256>>>(dD.as<unsigned int>(), length, dC.as<unsigned int>(), ncount,
                                                          dbad.as<unsigned int>());
    unsigned int bad = 0;
    EC_HIP(hipMemcpy(&bad, dbad.p, 4, hipMemcpyDeviceToHost));
    if (bad) {
        set_error("a component label D[i] is outside C[0..%llu)", (unsigned long long)ncount);
        return EC_ERR_ARG;
    }
    EC_HIP(hipMemcpy(C, dC.p, ncount * 4, hipMemcpyDeviceToHost));
    return EC_OK;
}

int ec_cg_vertices(const uint32_t *C, const uint32_t *offset, uint64_t ecount, uint32_t *cv, uint64_t ncv) {
    if (ecount && (!C || !offset || (ncv && !cv))) {
        set_error("null argument");
        return EC_ERR_ARG;
    }
    if (!ecount || !ncv) return EC_OK;
    EC_DEV(dC, ecount * 4);
    EC_DEV(dO, ecount * 4);
    EC_DEV(dcv, ncv * 4);
    EC_HIP(hipMemcpy(dC.p, C, ecount * 4, hipMemcpyHostToDevice));
    EC_HIP(hipMemcpy(dO.p, offset, ecount * 4, hipMemcpyHostToDevice));
    EC_HIP(hipMemcpy(dcv.p, cv, ncv * 4, hipMemcpyHostToDevice));
    k_cg_vertex<<<grid_for(ecount, 256), 256>>>(dC.as<unsigned int>(), dO.as<unsigned int>(), (unsigned int)ecount,
                                               dcv.as<unsigned int>(), (unsigned int)ncv);
    EC_HIP(hipMemcpy(cv, dcv.p, ncv * 4, hipMemcpyDeviceToHost));
    return EC_OK;
}

// calculateCircuitGraphEdgeData (cedge_count += per group) when cedge is null, else
// assignCircuitGraphEdgeData (cedge_count read-only: the reference passes it drv.In)
int ec_cg_edges_step(const void *ev, uint64_t vcount, const uint32_t *e, const uint32_t *D, const uint32_t *map,
                     uint64_t nmap, uint64_t ecount, const uint32_t *cedge_offset, uint32_t *cedge_count,
                     uint64_t ngroups, void *cedge, uint64_t cecount) {
    if ((vcount && !ev) || (ecount && (!e || !D)) || (nmap && !map) || !cedge_count ||
        (cedge && (!cedge_offset || (cecount && !cedge)))) {
        set_error("null argument");
        return EC_ERR_ARG;
    }
    if (!vcount || !ecount) return EC_OK;
    EC_DEV(dev, vcount * sizeof(EulerVertex));
    EC_DEV(de, ecount * 4);
    EC_DEV(dD, ecount * 4);
    EC_DEV(dmap, nmap * 4);
    EC_DEV(dcnt, ngroups * 4);
    EC_DEV(dper, vcount * 4);
    EC_HIP(hipMemcpy(dev.p, ev, vcount * sizeof(EulerVertex), hipMemcpyHostToDevice));
    EC_HIP(hipMemcpy(de.p, e, ecount * 4, hipMemcpyHostToDevice));
    EC_HIP(hipMemcpy(dD.p, D, ecount * 4, hipMemcpyHostToDevice));
    if (nmap) EC_HIP(hipMemcpy(dmap.p, map, nmap * 4, hipMemcpyHostToDevice));
    if (ngroups) EC_HIP(hipMemcpy(dcnt.p, cedge_count, ngroups * 4, hipMemcpyHostToDevice));
    if (!cedge) {  // calculate: the groups' counts added to cedge_count
        EC_DEV(dbad, 4);
        EC_HIP(hipMemset(dbad.p, 0, 4));
        k_cg_count<<<grid_for(vcount, 256), 256>>>(dev.as<EulerVertex>(), (unsigned int)vcount, de.as<unsigned int>(),
                                                  dD.as<unsigned int>(), dmap.as<unsigned int>(), (unsigned int)ecount,
                                                  (unsigned int)nmap, nullptr, dcnt.as<unsigned int>(),
                                                  (unsigned int)ngroups, dbad.as<unsigned int>());
        unsigned int bad = 0;
        EC_HIP(hipMemcpy(&bad, dbad.p, 4, hipMemcpyDeviceToHost));
        if (bad) {
            set_error("a circuit id is outside cedgeCount[0..%llu)", (unsigned long long)ngroups);
            return EC_ERR_ARG;
        }
        if (ngroups) EC_HIP(hipMemcpy(cedge_count, dcnt.p, ngroups * 4, hipMemcpyDeviceToHost));
        return EC_OK;
    }
    // assign: the candidates in sequential order, stably sorted by group
    k_cg_count<<<grid_for(vcount, 256), 256>>>(dev.as<EulerVertex>(), (unsigned int)vcount, de.as<unsigned int>(),
                                              dD.as<unsigned int>(), dmap.as<unsigned int>(), (unsigned int)ecount,
                                              (unsigned int)nmap, dper.as<unsigned int>(), nullptr, 0u, nullptr);
    EC_DEV(dbase, (vcount + 1) * 4);
    EC_CHECK(exscan_u32(dper.as<unsigned int>(), dbase.as<unsigned int>(), vcount));
    unsigned int last = 0, lastc = 0;
    EC_HIP(hipMemcpy(&last, dbase.as<unsigned int>() + vcount - 1, 4, hipMemcpyDeviceToHost));
    EC_HIP(hipMemcpy(&lastc, dper.as<unsigned int>() + vcount - 1, 4, hipMemcpyDeviceToHost));
    const uint64_t nc = (uint64_t)last + lastc;
    if (!nc) return EC_OK;
    EC_DEV(dkey, nc * 4);
    EC_DEV(dpos, nc * 4);
    EC_DEV(dkey2, nc * 4);
    EC_DEV(dpos2, nc * 4);
    EC_DEV(dcand, nc * 16);
    EC_DEV(doff, ngroups * 4);
    EC_DEV(dce, cecount * sizeof(CircuitEdge));
    k_cg_list<<<grid_for(vcount, 256), 256>>>(dev.as<EulerVertex>(), (unsigned int)vcount, de.as<unsigned int>(),
                                             dD.as<unsigned int>(), dmap.as<unsigned int>(), (unsigned int)ecount,
                                             (unsigned int)nmap, dbase.as<unsigned int>(), dkey.as<unsigned int>(),
                                             dpos.as<unsigned int>(), dcand.as<uint4>());
    size_t bytes = 0;
    EC_HIP(rocprim::radix_sort_pairs(nullptr, bytes, dkey.as<unsigned int>(), dkey2.as<unsigned int>(),
                                     dpos.as<unsigned int>(), dpos2.as<unsigned int>(), nc, 0, 32, (hipStream_t)0));
    EC_DEV(tmp, bytes);
    EC_HIP(rocprim::radix_sort_pairs(tmp.p, bytes, dkey.as<unsigned int>(), dkey2.as<unsigned int>(),
                                     dpos.as<unsigned int>(), dpos2.as<unsigned int>(), nc, 0, 32, (hipStream_t)0));
    if (ngroups) EC_HIP(hipMemcpy(doff.p, cedge_offset, ngroups * 4, hipMemcpyHostToDevice));
    if (cecount) EC_HIP(hipMemcpy(dce.p, cedge, cecount * sizeof(CircuitEdge), hipMemcpyHostToDevice));
    k_cg_assign<<<grid_for(nc, 256), 256>>>(dkey2.as<unsigned int>(), dpos2.as<unsigned int>(), (unsigned int)nc,
                                           dcand.as<uint4>(), doff.as<unsigned int>(), dcnt.as<unsigned int>(),
                                           (unsigned int)ngroups, dce.as<CircuitEdge>(), (unsigned int)cecount);
    if (cecount) EC_HIP(hipMemcpy(cedge, dce.p, cecount * sizeof(CircuitEdge), hipMemcpyDeviceToHost));
    return EC_OK;
}

}  // extern "C"
