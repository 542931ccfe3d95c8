// extended.h -- reads holding bytes other than A/C/G/T/N: soft-masked (lowercase) FASTA, IUPAC
// codes.  The reference keeps every such byte as an opaque symbol that is its own complement
// (referenceAssembler.py twin:7-10), splits a read on uppercase 'N' only (build:29) and
// extends a k-mer by the four uppercase bases only (fw / bw:16-22).
//
// Keys.  Each symbol present in the input gets a code of sb bits (A C G T = 0..3, the other
// bytes 4.. in byte order; sb = 4 / 5 / 8 for up to 16 / 32 / 256 symbols), a k-mer is the
// sb*k-bit code in a K128 (first symbol most significant) and must fit the HBM table's two
// 63-bit claim words: sb * k <= 126.  The complement of A C G T is 3 - c, of any other
// symbol the symbol itself, so the twin of a code is its symbol-reversed complement and
// canonical = min(code, twin).  Palindromes exist at odd k too (an opaque middle symbol);
// the count's "+2 for a palindrome" (build inserts it from both strands) covers any k.
//
// Links.  k_neighbors / k_succ apply get_contig_forward's rule as it is: |fw(x) in d| == 1,
// |bw(y) in d| == |fw(twin y) in d| == 1, y != twin(x).  With opaque symbols that rule is no
// longer symmetric: if x's FIRST symbol is opaque, x is not in bw(y), so x -> y can hold while
// y's single bw neighbour is another k-mer z (and z -> y holds too).  Such a one-way link has
// no twin link, y gets two predecessors, and walks from different starts overlap.  Components
// (weakly connected, over canonical ids) without a one-way link are the ordinary disjoint
// paths / cycles closed under twin and take the parallel ranking of graph.h unchanged; the
// few components with one (k_x_asym) are cut out of it and all_contigs:79-88 is emulated on
// them as written -- dict order, `done` set, get_contig's two walks -- one thread per
// component, entries pre-sorted by (component, first event) (k_x_emulate).  Their contigs are
// merged into the global order by their start's first event, and their GFA heads / tails
// follow the reference's dicts: a later contig with the same head k-mer replaces an earlier
// one (all_contigs:94-96).
#pragma once
#include "graph.h"

namespace ec {

struct XAlpha {
    uint32_t sb;        // bits per symbol
    uint32_t nsym;      // symbols in use (4 + opaque bytes present)
    uint8_t code[256];  // byte -> symbol code, 0xFF = 'N' (segment split)
    uint8_t dec[256];   // symbol code -> byte
};
__constant__ XAlpha c_xa;

// ---- 128-bit code algebra with sb-bit symbols ---------------------------------------------
__device__ inline K128 shl128(const K128 &x, uint32_t n) {  // 0 < n < 64
    K128 r;
    r.hi = (x.hi << n) | (x.lo >> (64 - n));
    r.lo = x.lo << n;
    return r;
}
__device__ inline K128 shr128(const K128 &x, uint32_t n) {  // 0 < n < 64
    K128 r;
    r.lo = (x.lo >> n) | (x.hi << (64 - n));
    r.hi = x.hi >> n;
    return r;
}
__device__ inline uint32_t sym_at(const K128 &x, uint32_t bit) {  // sb bits at bit
    const uint32_t m = (1u << c_xa.sb) - 1u;
    if (bit >= 64) return (uint32_t)(x.hi >> (bit - 64)) & m;
    unsigned long long v = x.lo >> bit;
    if (bit) v |= x.hi << (64 - bit);
    return (uint32_t)v & m;
}
__device__ inline uint32_t xcomp(uint32_t c) { return c < 4 ? 3u - c : c; }

struct OpsX {
    using K = K128;
    __device__ static inline K mask(int k) {
        const uint32_t bits = c_xa.sb * (uint32_t)k;  // <= 126
        K m;
        m.lo = bits >= 64 ? ~0ull : (1ull << bits) - 1;
        m.hi = bits > 64 ? (1ull << (bits - 64)) - 1 : 0ull;
        return m;
    }
    __device__ static inline K push(const K &x, uint32_t b, const K &m) {
        K r = shl128(x, c_xa.sb);
        r.lo |= b;
        r.lo &= m.lo;
        r.hi &= m.hi;
        return r;
    }
    __device__ static inline K twin(const K &x, int k) {
        const uint32_t sb = c_xa.sb;
        K r{0, 0};
        for (int i = 0; i < k; i++) {  // symbol i from the end becomes symbol i from the front
            const uint32_t c = xcomp(sym_at(x, sb * (uint32_t)i));
            r = shl128(r, sb);
            r.lo |= c;
        }
        return r;
    }
    __device__ static inline K twin_push(const K &tx, uint32_t b, int k) {
        K r = shr128(tx, c_xa.sb);
        const uint32_t bit = c_xa.sb * (uint32_t)(k - 1);
        const unsigned long long v = 3u - b;  // b is a base (fw / bw extend by A C G T only)
        if (bit >= 64) r.hi |= v << (bit - 64);
        else {
            r.lo |= v << bit;
            if (bit) r.hi |= v >> (64 - bit);
        }
        return r;
    }
    __device__ static inline uint32_t base(const K &x, int k, int i) { return sym_at(x, c_xa.sb * (uint32_t)(k - 1 - i)); }
    __device__ static inline uint32_t last(const K &x) { return (uint32_t)x.lo & ((1u << c_xa.sb) - 1u); }
    __device__ static inline char chr(uint32_t b) { return (char)c_xa.dec[b]; }
};

// ---- alphabet scan, prescan, count ----------------------------------------------------------
// the bytes present in the reads: a 256-bit mask (thread per read)
__global__ void __launch_bounds__(256) k_x_alphabet(const uint8_t *buf, const uint64_t *off, uint64_t nreads,
                                                    unsigned int *present) {
    __shared__ unsigned int m[8];
    if (threadIdx.x < 8) m[threadIdx.x] = 0;
    __syncthreads();
    for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < nreads; r += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t s = off[r], len = off[r + 1] - s;
        ByteReader rd(buf);
        for (uint64_t t = 0; t < len; t++) {
            const uint32_t c = rd(s + t);
            if (!(m[c >> 5] & (1u << (c & 31)))) atomicOr(&m[c >> 5], 1u << (c & 31));
        }
    }
    __syncthreads();
    if (threadIdx.x < 8 && m[threadIdx.x]) atomicOr(&present[threadIdx.x], m[threadIdx.x]);
}

// windows of read r in reference insertion order over sb-bit symbols (for_each_window_w with
// 'N' as the only separator)
template <typename Fn>
__device__ inline void for_each_window_x(ByteReader &rd, uint64_t s, uint64_t len, int k, uint64_t r, Fn &&fn) {
    const K128 mask = OpsX::mask(k);
    const uint32_t sb = c_xa.sb, top = sb * (uint32_t)(k - 1);
    uint32_t wb = 0;
    uint64_t p = 0;
    while (p < len) {
        uint64_t q = p;
        while (q < len && c_xa.code[rd(s + q)] != 0xFF) q++;
        if (q - p >= (uint64_t)k) {
            const uint32_t m = (uint32_t)(q - p - k + 1);
            K128 fwd{0, 0}, rc{0, 0};
            for (uint64_t t = p; t < q; t++) {
                const uint32_t b = c_xa.code[rd(s + t)];
                fwd = OpsX::push(fwd, b, mask);
                rc = shr128(rc, sb);
                const unsigned long long v = xcomp(b);
                if (top >= 64) rc.hi |= v << (top - 64);
                else {
                    rc.lo |= v << top;
                    if (top) rc.hi |= v >> (64 - top);
                }
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

__global__ void __launch_bounds__(256) k_x_prescan(const uint8_t *buf, const uint64_t *off, uint64_t nreads, int k,
                                                   unsigned int *hll, unsigned long long *npos) {
    __shared__ unsigned int reg[HLL_M];
    for (int i = threadIdx.x; i < HLL_M; i += blockDim.x) reg[i] = 0;
    __syncthreads();
    unsigned long long np = 0;
    for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < nreads; r += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t s = off[r], len = off[r + 1] - s;
        ByteReader rd(buf);
        for_each_window_x(rd, s, len, k, 0, [&](const K128 &f, const K128 &rc, uint64_t, uint64_t) {
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

// count (thread per read) into the wide HBM table, semantics of k_count_w
__global__ void __launch_bounds__(256) k_x_count(const uint8_t *buf, const uint64_t *off, uint64_t nreads, int k,
                                                 SlotW *table, uint64_t capmask, unsigned int *overflow) {
    for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < nreads; r += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t s = off[r], len = off[r + 1] - s;
        ByteReader rd(buf);
        for_each_window_x(rd, s, len, k, r, [&](const K128 &f, const K128 &rc, uint64_t ef, uint64_t er) {
            const bool pal = f == rc;  // (any k: an opaque middle symbol)
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

// all_contigs on a caller's dict of arbitrary k-byte strings (ec_assemble_from_kmers): as
// k_kmers_to_agg, symbols by c_xa.code ('N' is an opaque symbol here: no read to split)
__global__ void __launch_bounds__(256) k_x_kmers_to_agg(const char *chars, const unsigned int *counts, uint64_t n,
                                                        int k, AggW *out) {
    const K128 mask = OpsX::mask(k);
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < n; t += (uint64_t)gridDim.x * blockDim.x) {
        const char *x = chars + t * (uint64_t)k;
        K128 code{0, 0};
        for (int i = 0; i < k; i++) code = OpsX::push(code, c_xa.code[(unsigned char)x[i]], mask);
        const K128 tw = OpsX::twin(code, k);
        out[t] = RecOf<K128>::make(code < tw ? code : tw, code <= tw ? counts[t] : 0u,
                                   code <= tw ? (unsigned long long)t : ~0ull, tw <= code ? (unsigned long long)t : ~0ull);
    }
}

// ---- one-way links and their components -----------------------------------------------------
// asym[0] += links x -> y whose twin link twin(y) -> twin(x) is missing
__global__ void __launch_bounds__(256) k_x_asym(const uint8_t *upal, const unsigned int *succ, unsigned int N,
                                                unsigned int *nasym) {
    unsigned int c = 0;
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < N; t += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned int x = (unsigned int)t;
        if ((x & 1) && upal[x >> 1]) continue;
        const unsigned int y = succ[x];
        if (y == NONE32) continue;
        c += succ[twin_node(upal, y)] != twin_node(upal, x);
    }
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(nasym, c);
}

__global__ void __launch_bounds__(256) k_x_iota(unsigned int *x, uint64_t n) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < n; t += (uint64_t)gridDim.x * blockDim.x)
        x[t] = (unsigned int)t;
}

__device__ inline unsigned int uf_find(unsigned int *par, unsigned int x) {
    for (;;) {
        const unsigned int p = par[x];
        if (p == x) return x;
        const unsigned int g = par[p];
        if (g != p) par[x] = g;  // path halving (a racing store only writes another ancestor)
        x = p;
    }
}

__global__ void __launch_bounds__(256) k_x_uf_link(const uint8_t *upal, const unsigned int *succ, unsigned int N,
                                                   unsigned int *par) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < N; t += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned int x = (unsigned int)t;
        if ((x & 1) && upal[x >> 1]) continue;
        const unsigned int y = succ[x];
        if (y == NONE32) continue;
        unsigned int a = x >> 1, b = y >> 1;
        for (;;) {
            a = uf_find(par, a);
            b = uf_find(par, b);
            if (a == b) break;
            if (a < b) {
                const unsigned int t2 = a;
                a = b;
                b = t2;
            }
            if (atomicCAS(&par[a], a, b) == a) break;  // the larger root hooks under the smaller
        }
    }
}

// canonical id -> its component's root (into a separate array: path halving by other threads
// while flattening in place could overwrite a node's root with an intermediate ancestor); roots
// of components holding a one-way link get irr = 1
__global__ void __launch_bounds__(256) k_x_uf_flatten(unsigned int U, const unsigned int *par, unsigned int *root) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < U; t += (uint64_t)gridDim.x * blockDim.x) {
        unsigned int x = (unsigned int)t;
        for (unsigned int p = par[x]; p != x; p = par[x]) x = p;
        root[t] = x;
    }
}
__global__ void __launch_bounds__(256) k_x_mark_irr(const uint8_t *upal, const unsigned int *succ, unsigned int N,
                                                    const unsigned int *par, uint8_t *irr) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < N; t += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned int x = (unsigned int)t;
        if ((x & 1) && upal[x >> 1]) continue;
        const unsigned int y = succ[x];
        if (y != NONE32 && succ[twin_node(upal, y)] != twin_node(upal, x)) irr[par[x >> 1]] = 1;
    }
}
// per canonical id: in an irregular component?  Their successors are cut (saved in xsucc) so
// the parallel ranking sees singletons there; their dict entries are listed (event, node)
__global__ void __launch_bounds__(256) k_x_cut(const uint8_t *upal, unsigned int N, const unsigned int *par,
                                               const uint8_t *irr, uint8_t *xin, unsigned int *succ,
                                               unsigned int *xsucc, const unsigned long long *dfc,
                                               const unsigned long long *dft, unsigned long long *lk,
                                               unsigned int *lv, unsigned int *nl) {
    for (uint64_t t0 = blockIdx.x * (uint64_t)blockDim.x; t0 < N; t0 += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t t = t0 + threadIdx.x;
        const unsigned int x = (unsigned int)t;
        bool sel = false;
        if (t < N) {
            const bool in = irr[par[x >> 1]] != 0;
            if (!(x & 1)) xin[x >> 1] = in ? 1 : 0;
            xsucc[x] = succ[x];
            if (in) succ[x] = NONE32;
            sel = in && !((x & 1) && upal[x >> 1]);
        }
        const unsigned int i = wave_append(nl, sel);
        if (sel) {
            lk[i] = first_event(dfc, dft, x);
            lv[i] = x;
        }
    }
}
// sort key of the second pass: (component root, position in event order)
__global__ void __launch_bounds__(256) k_x_rekey(const unsigned int *lv, unsigned int n, const unsigned int *par,
                                                 unsigned long long *key) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        key[i] = ((unsigned long long)par[lv[i] >> 1] << 32) | i;
}

// k-mer x in fw(last)?  (get_contig:50: the walk from x closed a cycle)
__device__ inline bool x_in_fw(const K128 *dkey, unsigned int last, unsigned int x, int k) {
    const K128 cx = node_code<OpsX>(dkey, x, k), cl = node_code<OpsX>(dkey, last, k);
    const uint32_t b = OpsX::last(cx);
    return b < 4 && OpsX::push(cl, b, OpsX::mask(k)) == cx;
}

// get_contig_forward:59-77 over the saved successors: the walk from x, stopping at its own
// start or the start's twin; returns the last node and the node count (bad: longer than N,
// i.e. a cycle without the start -- the reference would never return)
__device__ inline unsigned int x_walk(const unsigned int *xsucc, unsigned int x, unsigned int tx, unsigned int N,
                                      unsigned int &n, unsigned int *bad) {
    unsigned int v = x;
    n = 1;
    for (;;) {
        const unsigned int s = xsucc[v];
        if (s == NONE32 || s == x || s == tx) break;
        v = s;
        if (++n > N) {
            atomicOr(bad, 1u);
            break;
        }
    }
    return v;
}

// all_contigs:79-88 on each irregular component, one thread per component (its entries are
// [a, b) of the sorted list, in dict order).  A start j records its node, m = 1 + the nodes
// of the walk from twin(x) the contig takes (1 if the forward walk closed a cycle) and the
// contig's node count; other entries get key NONE.
__global__ void __launch_bounds__(64) k_x_emulate(const unsigned int *lv, unsigned int n, const unsigned int *par,
                                                  const uint8_t *upal, const unsigned int *xsucc, const K128 *dkey,
                                                  int k, unsigned int N, const unsigned long long *dfc,
                                                  const unsigned long long *dft, uint8_t *done,
                                                  unsigned long long *skey, unsigned int *sval, unsigned int *xlen,
                                                  unsigned int *xm, unsigned int *nstarts, unsigned int *bad) {
    for (uint64_t a = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; a < n; a += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned int root = par[lv[a] >> 1];
        if (a && par[lv[a - 1] >> 1] == root) continue;  // not the first entry of its component
        unsigned int ns = 0;
        for (uint64_t j = a; j < n && par[lv[j] >> 1] == root; j++) {
            const unsigned int x = lv[j];
            skey[j] = NONE64;
            if (done[x]) continue;
            const unsigned int tx = twin_node(upal, x);
            unsigned int nf, nb;
            const unsigned int last = x_walk(xsucc, x, tx, N, nf, bad);
            x_walk(xsucc, tx, x, N, nb, bad);
            const bool cyc = x_in_fw(dkey, last, x, k);
            // done: every k-mer of the contig and its twin (all_contigs:85-87)
            unsigned int v = x;
            for (unsigned int i = 0; i < nf; i++) {
                done[v] = 1;
                done[twin_node(upal, v)] = 1;
                v = xsucc[v];
            }
            if (!cyc) {
                v = tx;
                for (unsigned int i = 0; i < nb; i++) {
                    done[v] = 1;
                    done[twin_node(upal, v)] = 1;
                    v = xsucc[v];
                }
            }
            skey[j] = first_event(dfc, dft, x);
            sval[j] = 0x80000000u | (unsigned int)j;
            xm[j] = cyc ? 1u : nb;  // nodes of the walk from twin(x) the contig takes, + 1
            xlen[j] = nf + xm[j] - 1;
            ns++;
        }
        if (ns) atomicAdd(nstarts, ns);
    }
}

// contig_to_string of an emulated contig: c = [twin(b_{m-1}) .. twin(b_1)] + c_fw, b = the
// walk from twin(x) (get_contig:52-55), or c_fw alone for a cycle.  Heads / tails: the
// reference's dicts keep the LAST contig with a given head k-mer (atomicMax of index + 1).
__global__ void __launch_bounds__(256) k_x_emit(const unsigned int *lv, const unsigned int *xlen, const unsigned int *xm,
                                                const unsigned int *xcid, const unsigned long long *skey, unsigned int n,
                                                const uint8_t *upal, const unsigned int *xsucc, const K128 *dkey, int k,
                                                const unsigned long long *coff, char *chars, unsigned int *cfirst,
                                                unsigned int *clast, unsigned int *xhead, unsigned int *xtail) {
    for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < n; j += (uint64_t)gridDim.x * blockDim.x) {
        if (skey[j] == NONE64) continue;
        const unsigned int x = lv[j], tx = twin_node(upal, x), len = xlen[j], ci = xcid[j];
        char *dst = chars + coff[ci];
        auto put = [&](unsigned int node, unsigned int pos) {
            const K128 code = node_code<OpsX>(dkey, node, k);
            if (pos == 0) {
                for (int i = 0; i < k; i++) dst[i] = OpsX::chr(OpsX::base(code, k, i));
                cfirst[ci] = node;
                atomicMax(&xhead[node], ci + 1);
            } else {
                dst[k - 1 + pos] = OpsX::chr(OpsX::last(code));
            }
            if (pos == len - 1) {
                clast[ci] = node;
                atomicMax(&xtail[twin_node(upal, node)], ci + 1);
            }
        };
        const unsigned int m = xm[j];
        unsigned int v = xsucc[tx];
        for (unsigned int i = 1; i < m; i++) {  // b_i -> position m - 1 - i, as its twin
            put(twin_node(upal, v), m - 1 - i);
            v = xsucc[v];
        }
        v = x;
        for (unsigned int i = 0; i + m - 1 < len; i++) {
            put(v, m - 1 + i);
            v = xsucc[v];
        }
    }
}
// the emulated contigs' heads / tails into the shared arrays (their nodes are disjoint from the
// ordinary contigs')
__global__ void __launch_bounds__(256) k_x_heads(unsigned int N, const unsigned int *xhead, const unsigned int *xtail,
                                                 unsigned int *headOf, unsigned int *tailOf) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < N; t += (uint64_t)gridDim.x * blockDim.x) {
        if (xhead[t]) headOf[t] = xhead[t] - 1;
        if (xtail[t]) tailOf[t] = xtail[t] - 1;
    }
}

}  // namespace ec
