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
#include "count_global.h"
#include "graph.h"

#include <rocprim/rocprim.hpp>

#include <algorithm>
#include <cmath>
#include <climits>
#include <cstring>
#include <cstddef>
#include <functional>
#include <type_traits>
#include <vector>

#include "count_part.h"
#include "count_v2.h"
#include "count_sk2.h"
#include "shard.h"
#include "compact.h"
#include "count_wide.h"
#include "hostin.h"
#include "join_w.h"
#include "extended.h"
#include "rank_tile.h"
#include "junction.h"
#include "join_local.h"

#include <atomic>
#include <chrono>
#include <dlfcn.h>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <thread>

namespace ec {

// ---------------------------------------------------------------------------------------
// host side
// device bytes the process's session buffers hold, and their high-water mark (ec_mem_stats:
// the per-rank HBM of the sharded and streaming paths is reported from these)
std::atomic<unsigned long long> g_hbm_held{0}, g_hbm_peak{0};
inline void hbm_account(long long d) {
    const unsigned long long now = g_hbm_held.fetch_add((unsigned long long)d) + (unsigned long long)d;
    unsigned long long pk = g_hbm_peak.load();
    while (now > pk && !g_hbm_peak.compare_exchange_weak(pk, now)) {
    }
}
bool memlog_on();

struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    // (spare: allocate that fraction more already the first time -- a size that varies from call
    // to call, like the gathered chain count)
    __attribute__((noinline)) int ensure(size_t bytes, unsigned int spare_div = 0) {
        if (bytes <= cap) return EC_OK;
        // a buffer that grows gets 1/8 of headroom: sizes that vary a little from call to call
        // (chain counts, received records) would otherwise reallocate -- ~1 ms a hipFree /
        // hipMalloc pair -- on every call that is a little larger than the last
        size_t want = std::max<size_t>(bytes, 256);
        if (cap) want += want / 8;
        else if (spare_div) want += want / spare_div;
        release();
        const auto t0 = std::chrono::steady_clock::now();
        if (hipMalloc(&p, want) != hipSuccess) {
            p = nullptr;
            set_error("hipMalloc(%zu) failed", want);
            return EC_ERR_NOMEM;
        }
        cap = want;
        hbm_account((long long)want);
        if (want >= (1ull << 30) && memlog_on()) {  // EULERHIP_MEMLOG=1: large buffers and their call sites
            // (lib+offset: llvm-symbolizer --obj=libeulerhip.so of the same build names the caller)
            Dl_info di{};
            void *ra = __builtin_return_address(0);
            const unsigned long off = dladdr(ra, &di) && di.dli_fbase ? (unsigned long)((char *)ra - (char *)di.dli_fbase) : 0ul;
            const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            fprintf(stderr, "[eulerhip mem] +%.2f GB (held %.2f GB) in %.1f ms at lib+0x%lx\n", want / 1e9,
                    g_hbm_held.load() / 1e9, ms, off);
        }
        return EC_OK;
    }
    template <typename T>
    T *as() const { return reinterpret_cast<T *>(p); }
    void release() {
        if (p) {
            const auto t0 = std::chrono::steady_clock::now();
            hipFree(p);
            hbm_account(-(long long)cap);
            if (cap >= (1ull << 30) && memlog_on())
                fprintf(stderr, "[eulerhip mem] -%.2f GB (held %.2f GB) in %.1f ms\n", cap / 1e9, g_hbm_held.load() / 1e9,
                        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
        }
        p = nullptr;
        cap = 0;
    }
};

// pinned host buffer (page-locked: D2H copies of the results run at full PCIe rate)
struct HostBuf {
    char *p = nullptr;
    size_t cap = 0, size = 0;
    int resize(size_t bytes) {
        size = bytes;
        if (bytes <= cap) return EC_OK;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        size_t want = std::max<size_t>(bytes + bytes / 4, 4096);
        if (hipHostMalloc(reinterpret_cast<void **>(&p), want, hipHostMallocDefault) != hipSuccess) {
            p = nullptr;
            size = 0;
            set_error("hipHostMalloc(%zu) failed", want);
            return EC_ERR_NOMEM;
        }
        cap = want;
        return EC_OK;
    }
    char *data() const { return p; }
    bool empty() const { return size == 0; }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = size = 0;
    }
};

template <typename T>
struct PinnedVec {  // std::vector-like view of a pinned HostBuf
    HostBuf b;
    size_t n = 0;
    int resize(size_t count) {
        n = count;
        return b.resize(count * sizeof(T));
    }
    T *data() const { return reinterpret_cast<T *>(b.p); }
    size_t size() const { return n; }
    bool empty() const { return n == 0; }
    T &operator[](size_t i) const { return data()[i]; }
    void release() {
        b.release();
        n = 0;
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
    DevBuf rid, rlist, nextR, PK, RK, PL, PM;
    DevBuf hist, ftot, cnt, offs, bstart, tot, recs, recs2, sub;
    DevBuf startOf, skeys, svals, skeys2, svals2, cidxOf, clen, coff, chars, cfirst, clast, headOf, tailOf;
    DevBuf lk, lcnt, tmp, dchars, dcounts;
    // results (host)
    bool have = false;
    int k = 0;
    ec_stats stats{};
    HostBuf h_chars;
    // the one-GPU results' characters in transfer form: 2-bit codes, 4 a byte (A C G T = 0..3;
    // every character of a standard-alphabet contig is one of them), nchars_host of them --
    // ec_copy_contigs widens them (ecoli10m_err: 38 MB of characters over PCIe took ~0.7 ms)
    bool chars_packed = false;
    uint64_t nchars_host = 0;
    // small device -> host reads (scalars, counts) go through this page-locked bounce buffer and
    // are delivered by host_sync: a pageable destination cost ~11 us more per round trip
    // (tools/micro/sync_lat.hip on MI355X: 27.2 vs 16.3 us), and a step has ~6 of them
    HostBuf bounce;
    struct Pend {
        void *dst;
        size_t off, n;
    };
    std::vector<Pend> pend;
    size_t bused = 0;
    hipEvent_t rd_ev = nullptr;  // host_wait: a read-back's event (created on first use)
    // the contig characters' early copy to host memory (phase_graph): its stream and events, and
    // the previous call's character total that sizes it
    hipStream_t ostream = nullptr;
    // oev[0] / [1]: emission done / characters copied; [2] contig offsets final; [3] link offsets final
    hipEvent_t oev[4] = {nullptr, nullptr, nullptr, nullptr};
    uint64_t last_nchars = 0;
    // bucket starts of the dense ids (k_skbucket3 marks each bucket's first id): the tile
    // ranking cuts its tiles there (k_tile_plan); valid from a super-k-mer count to its graph phase
    DevBuf bmark, rt_tb;
    bool bmark_ok = false;
    // the owner merge's marks (phase_merge_part): its solid count, 0 = none -- the partitioned
    // finish cuts its segment's tiles there when the segment is that merge's output
    uint64_t seg_marks = 0;
    // count_sk2's refine plan of the previous call: launched speculatively on the next call of
    // the same shape while the host reads the partition's scalars back (phase_count_sk2)
    struct SkSpec {
        bool valid = false;
        uint64_t G = 0, cap = 0, nreads = 0, read_base = 0, fcap = 0;
        uint32_t M = 0;
        int k = 0, bbits = 0;
    } skspec;
    PinnedVec<uint64_t> h_coff;  // result readbacks land in pinned host memory
    PinnedVec<uint64_t> h_loff;
    PinnedVec<int64_t> h_links;
    // the one-GPU results' links in transfer form (links_compact): per-side link counts as bytes
    // and the links as u32 (2 contig + end < 2^32) -- ec_copy_links widens them (ecoli10m_err:
    // 18 + 18 MB of u64 offsets and links after GFA cost ~0.65 ms of PCIe; now 2.2 + 9 MB)
    PinnedVec<uint8_t> h_lc8;
    PinnedVec<uint32_t> h_links32;
    bool links_compact = false;
    bool want_dict = false;
    hipEvent_t ev[2 * EC_NSTAGES] = {};
    hipEvent_t kev[2 * EC_NKERNELS] = {};
    bool kused[EC_NKERNELS] = {};
    bool sused[EC_NSTAGES] = {};
    bool events = false;
    bool timing = false;        // kernel events (EC_FLAG_TIMING or EC_FLAG_KERNEL_TIMING)
    bool stage_timing = false;  // stage events (EC_FLAG_TIMING)
    unsigned int n_dense = 0;  // dense k-mer arrays held by the session (shard / merge steps)
    bool stats_ok = false;     // ec_get_stats valid (any successful call)
    unsigned flags = 0;        // flags of the current call
    DevBuf ocnt, rbc, mbid, mbid2, midx, midx2, gcur, cwalk, ewalk, lc8;
    bool no_index = false;      // the call needs dense records only (shard count, owner merge)
    uint64_t shard_base = 0;    // ec_count_shard: global id of the shard's read 0 (added at export)
    // the super-k-mer fast path's read length of the last call on (offsets, reads): reused
    // without a host round trip -- k_skpart_w<., ., true> checks every read against it anyway
    const uint64_t *lc_off = nullptr;
    uint64_t lc_n = 0, lc_L = 0;
    bool filt = false;          // phase_count: k_bucket_filt (more distinct keys than LDS tables hold)
    int pmax = 1, pmin = 0;     // k_bucket_filt: 2^pmax part tables per bucket region
    float part_keys = 1400.0f;  // k_bucket_filt: target keys per part table
    DevBuf bnp;                 // k_bucket_filt: per-bucket part bits
    const unsigned long long *bbeg = nullptr, *bend = nullptr;  // launch_bucket: explicit bucket bounds
    uint32_t nseg = 1;          // ... as nseg record ranges per bucket
    DevBuf fcur, bb2;           // count_v2.h: final-bucket cursors, bucket bounds
    DevBuf nrec;                // graph.h NodeRec: successor + first event per node (k_walk)
    SolidIndex gidx{};          // index of the loaded solid set (ec_graph_load, k <= 32)
    SolidIndexW gidxw{};        // the same for k > 32
    bool graph_loaded = false;  // ec_graph_load held: ec_graph_links_part / ec_graph_finish valid
    // junction-partitioned graph (junction.h, round 5): the segment placed at its global ids
    // (ec_graph_place), no global set held; record / outbox scratch of the distributed join
    bool placed = false;
    uint64_t seg_lo = 0, seg_Ur = 0;
    DevBuf jrec, joid, jout, jseg, jcnt;
    DevBuf xrec;     // ec_merge_owned_from: the received records decoded
    DevBuf skm_rec, skm_ev, skm_end;  // k_skdedup: the merged records of the error-rich count
    DevBuf wcodes_tab;                // k_run_codes: each third-level table's first code dword
    HostBuf hmeta;   // ... and its per-source table, staged page-locked
    int owner_rule = 0;         // ec_session_set_owner_rule: 0 minimizer ranges (21 <= k <= 52), 1 key hash
    // ec_export_by_owner's owner ids / scanned chunk histogram of the last call, reused by a
    // following call with the same records, owners and rule (counts first, then the scatter)
    bool own_valid = false;
    int own_rule = 0, own_nowners = 0;
    unsigned int own_n = 0, own_nblk = 0;
    std::vector<unsigned int> own_hi;
    // host-input pipeline (ec_assemble_host / ec_assemble_packed_host, hostin.h): the reads are
    // copied H2D in chunks on cstream; pipe_upto(c) makes chunks .. c visible to the session
    // stream (event wait + unpack) -- the super-k-mer partition runs on each chunk's read groups
    // as they arrive, any other count path waits for all of them (pipe_all)
    hipStream_t cstream = nullptr;
    // a second copy stream (EULERHIP_COPY_STREAMS=2): chunks alternate between the two DMA queues.
    // One SDMA copy runs at half its idle rate while the count kernels run (r06_i trace); two
    // queues did not help (pipelined 5.22 / 5.22 ms on one, 5.23 / 5.95 on two: r06_m), so one
    hipStream_t cstream2 = nullptr;
    struct Pipe {
        bool active = false;
        bool packed = false;          // 2-bit codes (k_unpack2 + k_patch) or ASCII
        int nchunks = 0, done = 0;    // chunks made visible so far
        std::vector<uint64_t> blo, bhi;   // chunk c = bases [blo[c], bhi[c]) (multiples of 64 inside)
        std::vector<uint64_t> ravail;     // reads complete after chunk c
        std::vector<uint64_t> elo, ehi;   // its exceptions (packed)
        uint64_t first_len = 0;           // length of read 0 (the partition's M before any D2H)
        const uint32_t *codes = nullptr;  // device 2-bit codes
        const uint64_t *exc_pos = nullptr;
        const uint8_t *exc_byte = nullptr;
        uint8_t *ascii = nullptr;         // device reads (the count kernels' input)
        std::vector<hipEvent_t> ev;       // chunk copy events (created on demand, reused)
    } pipe;
    DevBuf p_codes, p_exc;
    // staged packed batches (ec_stage_packed_host / ec_assemble_staged): two slots, so the copy
    // of batch i + 1 runs on cstream while batch i is assembled; free_ev = the slot's last
    // reader (its assemble call) done on the session stream
    struct Staged {
        Pipe pipe;
        DevBuf codes, exc, off;
        hipEvent_t free_ev = nullptr;
        uint64_t nreads = 0, nbases = 0;
    } stg[2];
    int stg_head = 0, stg_n = 0;
    // extended alphabet (extended.h): its symbol table, and the one-way-link components'
    // union-find / cut / emulation buffers
    bool xalpha = false;
    XAlpha xa{};
    DevBuf x_par, x_irr, x_in, x_succ, x_done, x_lk, x_lv, x_lk2, x_lv2, x_len, x_m, x_cid, x_head, x_tail;
    // rank_tile.h: tile counts / bases, super list, its walk records, index map, path keys / ranks
    // join_local.h: per-key table words, table id ranges, foreign counts / offsets, flags
    DevBuf jl_kof, jl_rs, jl_re, jl_cnt, jl_off, jl_flag;
    DevBuf rpack;  // k_wbv's 2-bit copy of the reads (config 5's run codes gathered from it)
    DevBuf rt_tcnt, rt_tbase, rt_srec, rt_snrec, rt_sidx, rt_pks, rt_rks, rt_hasp, rt_lr;
    // Wyllie rounds the last converged super ranking needed + 1 (0: none yet, or it did not
    // converge): rank_supers_async queues that many instead of ceil(log2 N) + 2 -- a round after
    // convergence still costs its launch (~5 us; the headline needs ~18 of 26) -- and a shortfall
    // is caught by the convergence check that already follows (the ranking redone, host-checked)
    int spec_rounds = 0;
    DevBuf wbv;  // count_wide.h minimizer buckets: every window's minimizer
    // multi-GPU partitioned finish (ec_graph_chains_part ..): this rank's segment of oriented nodes
    uint64_t seg_n0 = 0, seg_n1 = 0;
    // a partitioned step called with a NULL output (ec_graph_place / chains_part / starts_part):
    // its records counted and held here until the matching ec_graph_*_copy writes them into a
    // buffer of the exact size (1: junction records, 2: super records, 3: start records)
    struct Pending {
        int kind = 0;
        uint64_t n = 0;
        unsigned int ntiles = 0;
        bool planned = false;
    } hold;
    SuperRec *chain_scr = nullptr;  // part_chains' tile records (st1, or a placed segment's jrec)
    unsigned int seg_nc = 0;     // contigs of the job (ec_graph_layout)
    uint64_t seg_nchars = 0;
    // the partitioned finish's transfer record (ec_graph_emit_runs / ec_graph_copy_runs):
    // chunk counts and scans, this rank's end records, the record's sizes
    DevBuf run_cnt, run_ends, run_dends;
    DevBuf rt_lb;                 // k_tile_chains' look-back status words (rank_tile.h TileLB)
    unsigned long long lb_epoch = 0;
    uint64_t run_nr = 0, run_nch = 0, run_nends = 0;
    bool runs_ready = false;
};

namespace {
constexpr size_t BOUNCE_CAP = 64 << 10, BOUNCE_MAX = 16 << 10;  // bytes; larger reads go direct

// queue a device -> host copy of n bytes to dst on st; dst is valid after host_sync(s, st)
int d2h(ec_session *s, void *dst, const void *src, size_t n, hipStream_t st) {
    if (!n) return EC_OK;
    const size_t off = (s->bused + 15) & ~size_t(15);
    if (n > BOUNCE_MAX || off + n > BOUNCE_CAP) {
        EC_HIP(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, st));
        return EC_OK;
    }
    if (!s->bounce.p) EC_CHECK(s->bounce.resize(BOUNCE_CAP));
    EC_HIP(hipMemcpyAsync(s->bounce.p + off, src, n, hipMemcpyDeviceToHost, st));
    s->pend.push_back({dst, off, n});
    s->bused = off + n;
    return EC_OK;
}

// wait for event ev (recorded after the d2h copies), then deliver the queued d2h reads: the
// stream may run on past it
int host_wait(ec_session *s, hipEvent_t ev) {
    const hipError_t e = hipEventSynchronize(ev);
    for (const auto &q : s->pend) std::memcpy(q.dst, s->bounce.p + q.off, q.n);
    s->pend.clear();
    s->bused = 0;
    if (e != hipSuccess) {
        set_error("HIP error %s", hipGetErrorString(e));
        return EC_ERR_HIP;
    }
    return EC_OK;
}

// wait for st, then deliver the queued d2h reads
int host_sync(ec_session *s, hipStream_t st) {
    const hipError_t e = hipStreamSynchronize(st);
    for (const auto &q : s->pend) std::memcpy(q.dst, s->bounce.p + q.off, q.n);
    s->pend.clear();
    s->bused = 0;
    if (e != hipSuccess) {
        set_error("HIP error %s", hipGetErrorString(e));
        return EC_ERR_HIP;
    }
    return EC_OK;
}
}  // namespace

namespace ec {

// all_contigs(d, k) from a caller's dict (referenceAssembler.py:79-111): entry i = (string,
// count) in dict order becomes an exchange record of its canonical key whose first event of
// the entry's orientation is i; a twin entry adds count 0 (build stores both strands with the
// same count).  bad gets the smallest entry index holding a byte outside ACGT.
template <typename Ops>
__global__ void __launch_bounds__(256) k_kmers_to_agg(const char *chars, const unsigned int *counts, uint64_t n, int k,
                                                      typename RecOf<typename Ops::K>::T *out, unsigned long long *bad) {
    using K = typename Ops::K;
    const K mask = Ops::mask(k);
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < n; t += (uint64_t)gridDim.x * blockDim.x) {
        const char *x = chars + t * (uint64_t)k;
        K code{};
        bool ok = true;
        for (int i = 0; i < k; i++) {
            const uint32_t b = base_code((unsigned char)x[i]);
            ok &= b < 4;
            code = Ops::push(code, b & 3u, mask);
        }
        if (!ok) atomicMin(bad, (unsigned long long)t);
        const K tw = Ops::twin(code, k);
        out[t] = RecOf<K>::make(code < tw ? code : tw, code <= tw ? counts[t] : 0u,
                                code <= tw ? (unsigned long long)t : ~0ull, tw <= code ? (unsigned long long)t : ~0ull);
    }
}
}  // namespace ec

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
    unsigned int ngath;  // phase_load_det: non-filler records of a gathered solid set
    unsigned long long nvisited;
    unsigned int maxlocal;
    unsigned int skew;
    unsigned int lens[4];  // k_upsweep: max read length, ~min read length (reads with windows), any slow-path read
    unsigned long long nrec;  // k_upsweep_sk: super-k-mer records
    unsigned int nasym, nxl, nxs;  // extended.h: one-way links, entries of their components, their starts
    unsigned int xbad;             // extended.h: a walk that never reaches its start again
    unsigned int wbv_long, wpad;     // k_wbv: a read of another length
    unsigned long long chains;       // k_tile_compact: the tile contraction's chain count
    unsigned int active[64];
};

int scan_u64(ec_session *s, const unsigned long long *in, unsigned long long *out, size_t n) {
    size_t bytes = 0;
    EC_HIP(rocprim::exclusive_scan(nullptr, bytes, in, out, 0ull, n, rocprim::plus<unsigned long long>(), s->stream));
    EC_CHECK(s->tmp.ensure(bytes));
    EC_HIP(rocprim::exclusive_scan(s->tmp.p, bytes, in, out, 0ull, n, rocprim::plus<unsigned long long>(), s->stream));
    return EC_OK;
}

int scan_excl_u32(ec_session *s, const unsigned int *in, unsigned int *out, size_t n) {
    size_t bytes = 0;
    EC_HIP(rocprim::exclusive_scan(nullptr, bytes, in, out, 0u, n, rocprim::plus<unsigned int>(), s->stream));
    EC_CHECK(s->tmp.ensure(bytes));
    EC_HIP(rocprim::exclusive_scan(s->tmp.p, bytes, in, out, 0u, n, rocprim::plus<unsigned int>(), s->stream));
    return EC_OK;
}

int scan_incl_u32(ec_session *s, const unsigned int *in, unsigned int *out, size_t n) {
    size_t bytes = 0;
    EC_HIP(rocprim::inclusive_scan(nullptr, bytes, in, out, n, rocprim::plus<unsigned int>(), s->stream));
    EC_CHECK(s->tmp.ensure(bytes));
    EC_HIP(rocprim::inclusive_scan(s->tmp.p, bytes, in, out, n, rocprim::plus<unsigned int>(), s->stream));
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

// make host-input chunks .. c visible on the session stream (no-op without a pipeline)
int pipe_upto(ec_session *s, int c) {
    auto &pp = s->pipe;
    if (!pp.active) return EC_OK;
    c = std::min(c, pp.nchunks - 1);
    if (pp.done > c) return EC_OK;
    const int first = pp.done;
    for (; pp.done <= c; pp.done++) EC_HIP(hipStreamWaitEvent(s->stream, pp.ev[pp.done], 0));
    // one unpack over the chunks made visible together (their ranges are contiguous)
    const uint64_t blo = pp.blo[first], bhi = pp.bhi[c], elo = pp.elo[first], ehi = pp.ehi[c];
    if (pp.packed && bhi > blo) {
        const uint64_t units = ((bhi + 15) >> 4) - (blo >> 4);
        k_unpack2<<<grid_for(units, 256, 16384), 256, 0, s->stream>>>(pp.codes, blo, bhi, pp.ascii);
        if (ehi > elo)
            k_patch<<<grid_for(ehi - elo, 256, 4096), 256, 0, s->stream>>>(pp.exc_pos, pp.exc_byte, elo, ehi,
                                                                           pp.ascii);
    }
    return EC_OK;
}
int pipe_all(ec_session *s) { return s->pipe.active ? pipe_upto(s, s->pipe.nchunks - 1) : EC_OK; }

inline void mark(ec_session *s, int idx) {
    if (s->stage_timing) {
        hipEventRecord(s->ev[idx], s->stream);
        if (idx & 1) s->sused[idx >> 1] = true;
    }
}
// kernel-level timing events: kernel id, 0 = before / 1 = after
inline void kmark(ec_session *s, int kid, int end) {
    if (s->timing) {
        hipEventRecord(s->kev[2 * kid + end], s->stream);
        if (end) s->kused[kid] = true;
    }
}

// elapsed times of the stage / kernel events recorded during this call (EC_FLAG_TIMING)
void collect_timing(ec_session *s) {
    if (!s->timing) return;
    hipStreamSynchronize(s->stream);
    for (int i = 0; i < EC_NSTAGES; i++) {
        float ms = 0;
        if (s->stage_timing && s->sused[i]) hipEventElapsedTime(&ms, s->ev[2 * i], s->ev[2 * i + 1]);
        s->stats.stage_ms[i] = ms;
    }
    for (int i = 0; i < EC_NKERNELS; i++) {
        float ms = 0;
        if (s->kused[i]) hipEventElapsedTime(&ms, s->kev[2 * i], s->kev[2 * i + 1]);
        s->stats.kernel_ms[i] = ms;
    }
}

// per-call setup shared by every entry point: argument checks, stats reset, timing events,
// zeroed device scalars
int begin_call(ec_session *s, int k, unsigned flags) {
    s->xalpha = false;  // (set by the extended-alphabet path, extended.h)
    s->hold.kind = 0;
    refresh_knobs();
    s->have = false;
    s->stats_ok = false;
    if (k < 1 || k > EC_MAX_K) {
        set_error("k=%d outside [1,%d]", k, EC_MAX_K);
        return EC_ERR_ARG;
    }
    EC_HIP(hipSetDevice(s->device));
    // (an earlier call that failed may have left a results copy in flight on the output stream)
    if (s->ostream) EC_HIP(hipStreamSynchronize(s->ostream));
    memset(&s->stats, 0, sizeof(s->stats));
    s->k = k;
    s->want_dict = (flags & EC_FLAG_WANT_DICT) != 0;
    s->flags = flags;
    s->shard_base = 0;
    s->own_valid = false;
    s->bmark_ok = false;
    s->seg_marks = 0;  // bucket marks of an earlier call never plan this call's tiles
    s->placed = false;
    const bool timing = (flags & (EC_FLAG_TIMING | EC_FLAG_KERNEL_TIMING)) != 0;
    s->stage_timing = (flags & EC_FLAG_TIMING) != 0;
    if (timing && !s->events) {
        for (auto &e : s->ev) EC_HIP(hipEventCreate(&e));
        for (auto &e : s->kev) EC_HIP(hipEventCreate(&e));
        s->events = true;
    }
    s->timing = timing;
    for (auto &u : s->kused) u = false;
    for (auto &u : s->sused) u = false;
    EC_CHECK(s->scal.ensure(sizeof(Scalars)));
    Scalars *dsc = s->scal.as<Scalars>();
    EC_HIP(hipMemsetAsync(dsc, 0, sizeof(Scalars), s->stream));
    EC_HIP(hipMemsetAsync(&dsc->bad, 0xFF, sizeof(unsigned long long), s->stream));
    return EC_OK;
}


// solid slots of an HBM table -> dense arrays (ids in table order); sets dsc->nsolid / ndistinct
template <typename SlotT, typename KeyT>
int compact_table(ec_session *s, SlotT *table, uint64_t cap, long long limit, KeyT *dkey) {
    hipStream_t st = s->stream;
    Scalars *dsc = s->scal.as<Scalars>();
    const unsigned int nblk = (unsigned int)((cap + COMPACT_CHUNK - 1) / COMPACT_CHUNK);
    EC_CHECK(s->rbc.ensure((size_t)nblk * 8 + 8));
    unsigned int *bc = s->rbc.as<unsigned int>(), *bs = bc + nblk;
    EC_HIP(hipMemsetAsync(&dsc->nsolid, 0, 4, st));
    EC_HIP(hipMemsetAsync(&dsc->ndistinct, 0, 8, st));
    k_compact_count<SlotT><<<nblk, 256, 0, st>>>(table, cap, limit, bc, &dsc->ndistinct);
    EC_CHECK(scan_incl_u32(s, bc, bs, nblk));
    k_compact_write<SlotT, KeyT><<<nblk, 256, 0, st>>>(table, cap, limit, bs, dkey, s->dcnt.as<unsigned int>(),
                                                      s->dfc.as<unsigned long long>(),
                                                      s->dft.as<unsigned long long>());
    k_compact_total<<<1, 1, 0, st>>>(bs, nblk, &dsc->nsolid);
    return EC_OK;
}


template <typename Src>
int launch_bucket(ec_session *s, Src src, unsigned nb, unsigned slots, long long limit, unsigned int *bmark = nullptr) {
    Scalars *dsc = s->scal.as<Scalars>();
    hipStream_t st = s->stream;
    // bucket b = records [bb[b], be[b]): the exact path's scanned starts, or the fixed-capacity
    // buckets of count_v2.h (s->bbeg / s->bend set)
    const unsigned long long *bb = s->bbeg ? s->bbeg : s->bstart.as<unsigned long long>();
    const unsigned long long *be = s->bbeg ? s->bend : s->bstart.as<unsigned long long>() + 1;
    const uint32_t ns = s->bbeg ? s->nseg : 1u;  // record ranges per bucket
    if (s->filt) {  // error-rich input: seen-twice filter + two half tables per bucket
        EC_CHECK(s->bnp.ensure(nb));
        k_bucket_filt<Src><<<nb, BUCKET_THREADS, 0, st>>>(
            src, bb, be, ns, limit, s->pmin, s->pmax, s->part_keys,
            s->dkey.as<unsigned long long>(),
            s->dcnt.as<unsigned int>(), s->dfc.as<unsigned long long>(), s->dft.as<unsigned long long>(),
            s->no_index ? nullptr : s->sub.as<SubSlot>(), s->bnp.as<uint8_t>(), &dsc->nsolid, &dsc->ndistinct,
            &dsc->overflow);
        return EC_OK;
    }
    if (slots == 2048)
        k_bucket<Src, 2048><<<nb, BUCKET_THREADS, 0, st>>>(
            src, bb, be, ns, limit, s->dkey.as<unsigned long long>(), s->dcnt.as<unsigned int>(),
            s->dfc.as<unsigned long long>(), s->dft.as<unsigned long long>(), s->no_index ? nullptr : s->sub.as<SubSlot>(), &dsc->nsolid,
            &dsc->ndistinct, &dsc->overflow, bmark);
    else
        k_bucket<Src, 4096><<<nb, BUCKET_THREADS, 0, st>>>(
            src, bb, be, ns, limit, s->dkey.as<unsigned long long>(), s->dcnt.as<unsigned int>(),
            s->dfc.as<unsigned long long>(), s->dft.as<unsigned long long>(), s->no_index ? nullptr : s->sub.as<SubSlot>(), &dsc->nsolid,
            &dsc->ndistinct, &dsc->overflow, bmark);
    return EC_OK;
}

// Bucket geometry of the partitioned path from the distinct estimate (shared by count_part.h's
// exact path and count_v2.h): 2^bbits final buckets of <= ~1100 keys, 2048- or 4096-slot LDS
// tables, or k_bucket_filt's seen-twice filter / part tables past ~2400 keys per bucket.
struct BucketPlan {
    bool part = false;  // partitioned counting applies at all (else the HBM table)
    bool filt = false;
    int pmax = 1;
    int bbits = 0;
    unsigned int slots = 2048;
};
BucketPlan plan_buckets(double est, long long limit, bool filt_ok) {
    constexpr int PMAX = 3;
    BucketPlan p;
    const double filt_max = limit >= 1 ? 32768.0 : PART_KEYS * (1 << PMAX);
    p.part = est / FINE <= 2400.0 || (filt_ok && est / FINE <= filt_max);
    p.filt = p.part && filt_ok && (est / FINE > 2400.0 || kn().force_filter);
    while (p.pmax < PMAX && est / FINE / (double)(1 << p.pmax) > PART_KEYS) p.pmax++;
    if (kn().filter_pmax) p.pmax = std::max(1, std::min(PMAX, kn().filter_pmax));
    while (p.bbits < FINE_BITS && est / (double)(1ull << p.bbits) > 1100.0) p.bbits++;
    p.slots = p.filt ? (2048u << p.pmax) : est / (double)(1ull << p.bbits) > 1100.0 ? 4096u : 2048u;
    return p;
}

// count_sk2.h: super-k-mer records for 21 <= k <= 32 (called by phase_count_v2 after its
// prescan).  done = false when the input does not qualify, the distinct estimate asks for the
// seen-twice filter, or a run / bucket / table outgrew its capacity: phase_count_v2 then counts
// with window records.
// validate: no k_prescan ran (phase_count_v2's fast path): M and npf come from the first read,
// the partition checks the input and counts the windows; *invalid = the input does not meet
// the prescan's conditions (the caller then takes the prescan path).
// workgroups of k_skpart_w<npf, w, val> the device runs at once (CUs x resident per CU)
static uint64_t skpart_slots(int npf, int w, bool val) {
    static thread_local int cache[3][SK_W_MAX + 1][2] = {};
    const int ni = npf == 4 ? 0 : npf == 7 ? 1 : 2;
    int &c = cache[ni][w][val];
    if (!c) {
        const void *fn = nullptr;
#define EC_SKF(NPF, W)                                                                                        \
    if (npf == NPF && w == W) fn = val ? (const void *)&k_skpart_w<NPF, W, true> : (const void *)&k_skpart_w<NPF, W, false>;
#define EC_SKF_W(W) EC_SKF(4, W) EC_SKF(7, W) EC_SKF(10, W)
        EC_SKF_W(7) EC_SKF_W(8) EC_SKF_W(9) EC_SKF_W(10) EC_SKF_W(11) EC_SKF_W(12)
        EC_SKF_W(13) EC_SKF_W(14) EC_SKF_W(15) EC_SKF_W(16) EC_SKF_W(17) EC_SKF_W(18)
#undef EC_SKF_W
#undef EC_SKF
        int dev = 0, ncu = 0, per = 0;
        if (!fn || hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fn, PT_THREADS, 0) != hipSuccess || per < 1)
            return 1;
        c = ncu * per;
    }
    return (uint64_t)c;
}

int phase_count_sk2(ec_session *s, const uint8_t *d_reads, const uint64_t *d_off, uint64_t nreads,
                    uint64_t read_base, int k, long long limit, uint32_t M, uint64_t G, uint64_t gsize, uint64_t P,
                    int npf, unsigned int &U, SolidIndex &sidx, bool &done, bool validate = false,
                    bool *invalid = nullptr) {
    done = false;
    if (invalid) *invalid = false;
    if (k >= SK_MIN_K && k <= 32) {
        // read groups: a multiple of the workgroups resident at once when there are more tiles
        // than that (2030 groups of 77 tiles on 768 slots ran 2.64 waves of workgroups, the last
        // one a third idle; 1536 of 102 tiles run 2 full ones), at most RF_MAX_RUNS (k_skrefine)
        const uint64_t ntiles = (nreads + 63) / 64, slots = skpart_slots(npf, k - SK_M + 1, validate);
        uint64_t g = std::max<uint64_t>(1, std::min<uint64_t>(ntiles, RF_MAX_RUNS));
        if (g > slots && !kn().no_slot_groups) g = g / slots * slots;
        gsize = ((ntiles + g - 1) / g) * 64;
        G = (nreads + gsize - 1) / gsize;
    }
    if (k < SK_MIN_K || k > 32 || M > 256 || gsize * M >= (1ull << 24) || (read_base + nreads) * 2 * M >= (1ull << 32) ||
        kn().no_sk2)
        return EC_OK;
    hipStream_t st = s->stream;
    Scalars *dsc = s->scal.as<Scalars>();
    Scalars hsc;
    auto reset = [&]() -> int {  // scalars as phase_count_v2 expects them after its prescan
        if (validate) {  // as begin_call left them: the prescan runs next
            EC_HIP(hipMemsetAsync(dsc, 0, sizeof(Scalars), st));
            EC_HIP(hipMemsetAsync(&dsc->bad, 0xFF, sizeof(unsigned long long), st));
            return EC_OK;
        }
        EC_HIP(hipMemsetAsync(&dsc->overflow, 0, sizeof(unsigned int), st));
        EC_HIP(hipMemsetAsync(&dsc->skew, 0, sizeof(unsigned int), st));
        EC_HIP(hipMemsetAsync(&dsc->nsolid, 0, sizeof(unsigned int), st));
        EC_HIP(hipMemsetAsync(&dsc->ndistinct, 0, sizeof(unsigned long long), st));
        return EC_OK;
    };
    const MinCfg mc = sk_cfg(k);
    constexpr uint64_t C = 1ull << SK2_CBITS;
    // records per read ~ 2 M / (w + 1) + 1 on random sequence; 40 % headroom per run
    const double per_read = 2.0 * M / (mc.w + 1) + 2.0;
    const uint64_t cap = (uint64_t)(gsize * per_read * 1.4 / C) + 256;
    EC_CHECK(s->recs.ensure((C * G * cap + SK2_ECAP_W) * 16));  // + the spill records
    EC_CHECK(s->cnt.ensure(C * G * 4));
    EC_CHECK(s->hll.ensure(G * (1 << HLL_REG_BITS)));
    EC_CHECK(s->ftot.ensure((1 << HLL_REG_BITS) * 4));
    uint4 *recs = s->recs.as<uint4>();
    const uint32_t smask = P >= (1ull << 26) ? 255u : 0u;
    unsigned int *hreg = s->ftot.as<unsigned int>();
    EC_HIP(hipMemsetAsync(&dsc->nrec, 0, sizeof(unsigned long long), st));
    mark(s, 2 * EC_STAGE_COUNT);
    kmark(s, 1, 0);
#define EC_SKPART_WV(NPF, W, VAL)                                                                             \
    k_skpart_w<NPF, W, VAL><<<lgb - lga, PT_THREADS, 0, st>>>(                                                   \
        d_reads, d_off, nreads, mc, M, gsize, (uint32_t)G, cap, smask, recs, s->cnt.as<unsigned int>(),          \
        s->hll.as<uint8_t>(), &dsc->nrec, &dsc->overflow, &dsc->lens[2], &dsc->npos, lga, elim)
#define EC_SKPART_W(NPF, W)            \
    if (validate)                      \
        EC_SKPART_WV(NPF, W, true);    \
    else                               \
        EC_SKPART_WV(NPF, W, false)
#define EC_SKPART_NPF(W)              \
    if (npf == 4) EC_SKPART_W(4, W);  \
    else if (npf == 7) EC_SKPART_W(7, W); \
    else EC_SKPART_W(10, W)
    // register-block minima for every window width of 21 <= k <= 32 (w = k - 14; an LDS-ring
    // sliding minimum measured 2.19 against 1.60 ms at k = 31).
    // Host input (s->pipe): one launch per arrived chunk, over the groups whose reads it completes
    const bool chunked = s->pipe.active && s->pipe.done < s->pipe.nchunks;
    if (!chunked) EC_CHECK(pipe_all(s));
    unsigned lga = 0, lgb = (unsigned)G;
    // entries a partition wave buffers (EULERHIP_SK2_ELIM: fewer, to test the overflow path)
    const uint32_t elim = kn().sk2_elim >= 128 ? (uint32_t)std::min(kn().sk2_elim, SK2_ECAP_W) : (uint32_t)SK2_ECAP_W;
    for (int pc = chunked ? 0 : s->pipe.nchunks; ; pc++) {
      if (chunked) {
        if (pc >= s->pipe.nchunks) break;
        lgb = pc + 1 == s->pipe.nchunks ? (unsigned)G : (unsigned)std::min<uint64_t>(G, s->pipe.ravail[pc] / gsize);
        if (lgb <= lga) continue;
        EC_CHECK(pipe_upto(s, pc));
      }
      {
        switch (mc.w) {
            case 7: EC_SKPART_NPF(7); break;
            case 8: EC_SKPART_NPF(8); break;
            case 9: EC_SKPART_NPF(9); break;
            case 10: EC_SKPART_NPF(10); break;
            case 11: EC_SKPART_NPF(11); break;
            case 12: EC_SKPART_NPF(12); break;
            case 13: EC_SKPART_NPF(13); break;
            case 14: EC_SKPART_NPF(14); break;
            case 15: EC_SKPART_NPF(15); break;
            case 16: EC_SKPART_NPF(16); break;
            case 17: EC_SKPART_NPF(17); break;
            default: EC_SKPART_NPF(18); break;  // k = 32
        }
      }
      if (!chunked) break;
      lga = lgb;
    }
#undef EC_SKPART_NPF
#undef EC_SKPART_W
#undef EC_SKPART_WV
    kmark(s, 1, 1);
    EC_HIP(hipMemsetAsync(hreg, 0, (1 << HLL_REG_BITS) * 4, st));
    k_hll_merge<<<dim3((1 << HLL_REG_BITS) / 256, TOT_SLICES), 256, 0, st>>>(s->hll.as<uint8_t>(), G, hreg);
    k_hll_final<<<1, 1024, 0, st>>>(hreg, HLL_REG_BITS, &dsc->est);
    EC_CHECK(d2h(s, &hsc, dsc, sizeof(Scalars), st));
    // ---- refine into fixed-capacity final buckets (launched below, or here on speculation) ----
    // a bucket gathers whole minimizers (each ~coverage records): ~13 % spread at the headline
    // size (62 minimizers a bucket), so twice the mean: fcap = 2 NR / buckets + 1024
    auto launch_refine = [&](int bb, uint64_t fc) -> int {
        const uint64_t nb = 1ull << bb;
        EC_CHECK(s->recs2.ensure(nb * fc * 16));
        EC_CHECK(s->fcur.ensure(nb * 8));
        EC_CHECK(s->bb2.ensure(nb * 16));
        EC_HIP(hipMemsetAsync(s->fcur.p, 0, nb * 8, st));
        unsigned rs = 8;
        if (kn().refine_rs) rs = (unsigned)std::max(1, kn().refine_rs);
        rs = (unsigned)std::min<uint64_t>(rs, G);
        kmark(s, 4, 0);
        k_skrefine<<<dim3((unsigned)C, rs), BUCKET_THREADS, 0, st>>>(recs, s->cnt.as<unsigned int>(), (uint32_t)G, cap,
                                                                      bb, s->recs2.as<uint4>(), fc,
                                                                      s->fcur.as<unsigned long long>(), &dsc->skew, M,
                                                                      gsize, read_base);
        kmark(s, 4, 1);
        unsigned long long *b0 = s->bb2.as<unsigned long long>();
        k_fixed_bounds<<<grid_for(nb, 256), 256, 0, st>>>(s->fcur.as<unsigned long long>(), nb, fc, b0, b0 + nb);
        return EC_OK;
    };
    // the previous call's plan for an input of this shape (a stream of equal batches, the bench's
    // steps) runs the refine while the host waits for the scalars -- the host's wake-up and the
    // plan below overlap the refine instead of idling the device (~40 us a call); a plan that
    // turns out different launches the refine again (it only writes recs2 / fcur / bb2)
    const auto sp = s->skspec;
    const bool spec = sp.valid && sp.G == G && sp.cap == cap && sp.nreads == nreads && sp.read_base == read_base &&
                      sp.M == M && sp.k == k && !chunked && kn().no_spec == 0;
    s->skspec.valid = false;
    if (spec) {
        if (!s->rd_ev) EC_HIP(hipEventCreateWithFlags(&s->rd_ev, hipEventDisableTiming));
        EC_HIP(hipEventRecord(s->rd_ev, st));
        EC_CHECK(launch_refine(sp.bbits, sp.fcap));
        EC_CHECK(host_wait(s, s->rd_ev));
    } else {
        EC_CHECK(host_sync(s, st));
    }
    const bool verbose = kn().verbose;
    if (validate) {
        if (hsc.lens[2]) {  // a read of another length, a byte outside ACGT, an oversized tile
            if (verbose) fprintf(stderr, "count_sk2: input needs the prescan\n");
            if (invalid) *invalid = true;
            return reset();
        }
        P = hsc.npos;
    }
    if (hsc.overflow) {  // a run outgrew its capacity
        if (verbose) fprintf(stderr, "count_sk2: partition run overflow (cap %llu)\n", (unsigned long long)cap);
        return reset();
    }
    const double est = hsc.est * (smask + 1.0);
    BucketPlan plan = plan_buckets(est, limit, !kn().no_filter);
    // error-rich input (the estimate asks for the seen-twice filter): super-k-mer buckets behind
    // the filter (k_skbucket_filt) while a bucket's distinct keys stay within its 2^16 filter
    // cells (limit >= 1); otherwise window records with count_part.h's filter
    const bool skfilt = plan.part && plan.filt && limit >= 1 && kn().sk_filt != 0 &&
                        est / (double)(1ull << SK2_BBITS) <= 16000.0;
    if (!plan.part || (plan.filt && !skfilt)) return reset();
    // up to 2^SK2_BBITS buckets of <= 1100 estimated keys (2048-slot tables: two workgroups per
    // CU).  Measured: 16384 buckets of 1024 slots (three workgroups per CU) were not faster, and
    // small tables need lds_insert to count claims after the CAS (reservations of up to 1024
    // racing lanes overshoot), which cost 8 % in every table
    // (<= 800 estimated keys a bucket: the estimate is +-3 %, and a bucket past ~1100 keys makes
    // both the count and the graph phase's probes measurably slower -- headline A/B 8192 against
    // 4096 buckets: k_skbucket 1.65 / 2.37 ms, links 0.56 / 1.07 ms)
    int bbits = SK2_CBITS;
    // k_skbucket3 (three workgroups per CU, 1024-slot tables) while its buckets stay at <= 380
    // estimated keys; larger inputs take k_skbucket's 2048- / 4096-slot tables
    const bool b3 = !skfilt && !kn().no_skb3 && est / (double)(1ull << SK2_BBITS) <= 380.0;
    const double per_bucket = b3 ? 380.0 : 800.0;
    while (bbits < SK2_BBITS && est / (double)(1ull << bbits) > per_bucket) bbits++;
    if (skfilt) bbits = SK2_BBITS;
    plan.bbits = bbits;
    plan.slots = skfilt ? 2048u : b3 ? 1024u : est / (double)(1ull << bbits) > 1100.0 ? 4096u : 2048u;
    const uint64_t Bk = 1ull << bbits;
    const uint64_t NR = hsc.nrec;
    uint64_t fcap = NR * 2 / Bk + 1024;
    if (spec && sp.bbits == bbits && sp.fcap >= fcap && sp.fcap <= fcap + fcap / 8) {
        fcap = sp.fcap;  // the speculative refine stands
    } else {
        if (spec && verbose) fprintf(stderr, "count_sk2: refine plan changed (bits %d -> %d), refined again\n", sp.bbits, bbits);
        fcap += fcap / 16;  // (headroom: the next call of this shape keeps the plan)
        EC_CHECK(launch_refine(bbits, fcap));
    }
    s->skspec.valid = true;
    s->skspec.G = G;
    s->skspec.cap = cap;
    s->skspec.nreads = nreads;
    s->skspec.read_base = read_base;
    s->skspec.fcap = fcap;
    s->skspec.M = M;
    s->skspec.k = k;
    s->skspec.bbits = bbits;
    unsigned long long *bbeg = s->bb2.as<unsigned long long>(), *bend = bbeg + Bk;
    mark(s, 2 * EC_STAGE_COUNT + 1);

    // ---- super-k-mers -> bucket tables ----------------------------------------------------------
    mark(s, 2 * EC_STAGE_COMPACT);
    const uint64_t umax = Bk * plan.slots;
    EC_CHECK(s->dkey.ensure(umax * 8));
    EC_CHECK(s->dcnt.ensure(umax * 4));
    EC_CHECK(s->dfc.ensure(umax * 8));
    EC_CHECK(s->dft.ensure(umax * 8));
    EC_CHECK(s->sub.ensure(umax * sizeof(SubSlot)));
    kmark(s, 2, 0);
    const double inv_m = 1.0 / M;
    // records deduplicated per bucket before their windows are rolled out (k_skbucket3 /
    // k_skbucket: 10x fewer k-mer inserts than one per record window on the headline)
#define EC_SKBUCKET_ARGS                                                                                     \
    s->recs2.as<uint4>(), bbeg, bend, k, M, inv_m, limit, s->dkey.as<unsigned long long>(),                    \
        s->dcnt.as<unsigned int>(), s->dfc.as<unsigned long long>(), s->dft.as<unsigned long long>(),          \
        s->no_index ? nullptr : s->sub.as<SubSlot>(), &dsc->nsolid, &dsc->ndistinct, &dsc->overflow
#define EC_SKBUCKET(SLOTS, RS, EVEN) \
    k_skbucket<SLOTS, RS, 1, EVEN><<<(unsigned)Bk, BUCKET_THREADS, 0, st>>>(EC_SKBUCKET_ARGS, dbg)
    // EULERHIP_SK2_STATS: distinct records, flushes and windows rolled out (stderr)
    bool b3_marked = false;
    unsigned long long *dbg = nullptr;
    if (kn().sk2_stats) {
        EC_CHECK(s->tmp.ensure(128));
        dbg = s->tmp.as<unsigned long long>();
        EC_HIP(hipMemsetAsync(dbg, 0, 128, st));
    }
    if (skfilt) {
        constexpr int NTF = 512;
        // (the table takes up to 2047 keys; the prediction runs ~10 % high.  ecoli10m_err's
        // fullest bucket: 1525 predicted, 1485 inserted)
        const unsigned int max_keys = kn().skf_keys > 0 ? (unsigned int)kn().skf_keys : 1900u;
        // (round 4 measured a record merge inside the filter kernel on ecoli10m_err: its 1535-entry
        // tables filled -- up to 915 records a bucket rejected -- and its 131 KB of LDS held one
        // workgroup per CU: compact 8.26 ms against 7.75 without it; round 5 merges in a kernel
        // of its own, k_skdedup, EULERHIP_SKF_MERGE=0 the filter alone.
        // No tile planning here: measured on ecoli10m_err the planned tiles left more chains,
        // 11.2 M against 10.9 M -- its graph is cut by error branches, not by tile edges)
        unsigned int *bm = nullptr;
        if (kn().skf_merge != 0) {
            // the bucket's duplicate records merged first (k_skdedup), the filter on the merged ones
            // (bucket b's merged records at its refine region [bbeg[b], ..): Bk x fcap records)
            EC_CHECK(s->skm_rec.ensure(Bk * fcap * sizeof(uint4)));
            EC_CHECK(s->skm_ev.ensure(Bk * fcap * sizeof(uint2)));
            EC_CHECK(s->skm_end.ensure(Bk * 8));
            uint4 *mrec = s->skm_rec.as<uint4>();
            uint2 *mev = s->skm_ev.as<uint2>();
            unsigned long long *mend = s->skm_end.as<unsigned long long>();
            const unsigned int claim_cap = kn().sk2_claim > 0 ? (unsigned int)kn().sk2_claim : ~0u;
            // (4096-entry tables, 1024 threads, one workgroup per CU: compact 2.87-2.92 ms on
            // ecoli10m_err against 3.03-3.06 with 2560 entries and two workgroups per CU)
            if (kn().skf_merge != 2)
                k_skdedup<4096, 1024><<<(unsigned)Bk, 1024, 0, st>>>(s->recs2.as<uint4>(), bbeg, bend, k, M, inv_m, mrec,
                                                                     mev, mend, claim_cap, dbg);
            else
                k_skdedup<2560, 512><<<(unsigned)Bk, 512, 0, st>>>(s->recs2.as<uint4>(), bbeg, bend, k, M, inv_m, mrec,
                                                                   mev, mend, claim_cap, dbg);
#define EC_SKF_MERGED_ARGS                                                                                   \
    mrec, bbeg, mend, k, M, inv_m, limit, s->dkey.as<unsigned long long>(), s->dcnt.as<unsigned int>(),      \
        s->dfc.as<unsigned long long>(), s->dft.as<unsigned long long>(),                                    \
        s->no_index ? nullptr : s->sub.as<SubSlot>(), &dsc->nsolid, &dsc->ndistinct, &dsc->overflow, max_keys, \
        dbg, bm, mev
            if (k & 1)
                k_skbucket_filt<2048, NTF, false, true><<<(unsigned)Bk, NTF, 0, st>>>(EC_SKF_MERGED_ARGS);
            else
                k_skbucket_filt<2048, NTF, true, true><<<(unsigned)Bk, NTF, 0, st>>>(EC_SKF_MERGED_ARGS);
#undef EC_SKF_MERGED_ARGS
        } else if (k & 1)
            k_skbucket_filt<2048, NTF, false><<<(unsigned)Bk, NTF, 0, st>>>(EC_SKBUCKET_ARGS, max_keys, dbg, bm);
        else
            k_skbucket_filt<2048, NTF, true><<<(unsigned)Bk, NTF, 0, st>>>(EC_SKBUCKET_ARGS, max_keys, dbg, bm);
        b3_marked = bm != nullptr;
    } else if (plan.slots == 1024) {
        constexpr int NT3 = 512;
        const unsigned int claim_cap = kn().sk2_claim > 0 ? (unsigned int)kn().sk2_claim : ~0u;
        unsigned int *bm = nullptr;
        if (kn().tile_plan != 0) {  // (bucket starts for the tile ranking: one bit per dense id)
            const size_t words = umax / 32 + 2;
            EC_CHECK(s->bmark.ensure(words * 4));
            EC_HIP(hipMemsetAsync(s->bmark.p, 0, words * 4, st));
            bm = s->bmark.as<unsigned int>();
        }
        if (k & 1)
            k_skbucket3<1024, 1664, NT3, false><<<(unsigned)Bk, NT3, 0, st>>>(EC_SKBUCKET_ARGS, dbg, claim_cap, bm);
        else
            k_skbucket3<1024, 1664, NT3, true><<<(unsigned)Bk, NT3, 0, st>>>(EC_SKBUCKET_ARGS, dbg, claim_cap, bm);
        b3_marked = bm != nullptr;
    } else if (plan.slots == 2048) {
        if (k & 1) EC_SKBUCKET(2048, 3072, false);
        else EC_SKBUCKET(2048, 3072, true);
    } else {
        if (k & 1) EC_SKBUCKET(4096, 2048, false);
        else EC_SKBUCKET(4096, 2048, true);
    }
#undef EC_SKBUCKET
#undef EC_SKBUCKET_ARGS
    if (dbg) {
        unsigned long long h[16];
        EC_CHECK(d2h(s, h, dbg, 128, st));
        EC_CHECK(host_sync(s, st));
        const double nw = (double)Bk * (BUCKET_THREADS / 64);  // waves
        if (skfilt)
            fprintf(stderr, "k_skbucket_filt: %llu buckets: max distinct est %llu, max predicted inserts %llu, max "
                            "seen-twice cells %llu, max records %llu; refused by the predictor %llu, tables filled "
                            "%llu, most keys inserted %llu; most merged records %llu, most past the claim cap %llu, "
                            "merged records %llu of %llu\n",
                    (unsigned long long)Bk, h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], h[8], h[9],
                    (unsigned long long)NR);
        if (plan.slots == 1024)
            fprintf(stderr, "k_skbucket3: %llu buckets, most distinct records in a bucket %llu\n",
                    (unsigned long long)Bk, h[3]);
        fprintf(stderr, "k_skbucket per wave (shader clocks): records phase canon %.0f probe %.0f (%.1f iterations) "
                        "post %.0f barrier %.0f over %.1f rounds; roll-out %.0f barrier %.0f\n",
                h[8] / nw, h[9] / nw, h[11] / nw, h[10] / nw, h[12] / nw, h[13] / nw, h[14] / nw, h[15] / nw);
        fprintf(stderr, "k_skbucket: %llu records, %llu distinct in %llu flushes (%.2f / bucket), %llu windows rolled "
                        "(positions %llu); block-us: init %.0f records %.0f sort %.0f roll-out %.0f finish %.0f\n",
                (unsigned long long)NR, h[0], h[1], (double)h[1] / Bk, h[2], (unsigned long long)P, h[3] / 100.0,
                h[4] / 100.0, h[5] / 100.0, h[6] / 100.0, h[7] / 100.0);
    }
    kmark(s, 2, 1);
    mark(s, 2 * EC_STAGE_COMPACT + 1);
    EC_CHECK(d2h(s, &hsc, dsc, sizeof(Scalars), st));
    EC_CHECK(host_sync(s, st));
    if (hsc.overflow || hsc.skew) {  // a final bucket or an LDS table overflowed
        if (verbose)
            fprintf(stderr, "count_sk2: %s overflow (%llu buckets, %u slots, est %.0f, fcap %llu)\n",
                    hsc.skew ? "final bucket" : "table", (unsigned long long)Bk, plan.slots, est,
                    (unsigned long long)fcap);
        s->stats.table_retries++;
        return reset();
    }
    done = true;
    s->bmark_ok = b3_marked;
    s->stats.n_positions = P;
    s->stats.n_distinct_est = (uint64_t)llround(est);
    s->stats.record_bytes = 16;
    s->stats.n_records = NR;
    s->stats.count_path = EC_PATH_PARTITIONED;
    s->stats.count_variant = 3;
    s->stats.n_buckets = (uint32_t)Bk;
    s->stats.table_capacity = umax;
    sidx = SolidIndex{};
    sidx.sub = s->sub.as<SubSlot>();
    sidx.bbits = bbits;
    sidx.slots = plan.slots;
    sidx.sk = 1;
    sidx.mc = mc;
    sidx.npb = nullptr;
    U = hsc.nsolid;
    s->stats.n_distinct = hsc.ndistinct;
    s->stats.n_solid = U;
    if (2ull * U >= (unsigned long long)CYC) {
        set_error("too many solid k-mers (%u) for 31-bit node ids", U);
        return EC_ERR_CAPACITY;
    }
    return EC_OK;
}

// count_v2.h: the partitioned count of N-free reads of one length without the histogram
// upsweep.  ok = false (and nothing decided) when the input does not qualify or a run / final
// bucket outgrew its fixed capacity: phase_count then takes count_part.h's exact path.
int phase_count_v2(ec_session *s, const uint8_t *d_reads, const uint64_t *d_off, uint64_t nreads, uint64_t read_base,
                   int k, long long limit, bool allow_sk2, unsigned int &U, SolidIndex &sidx, bool &ok) {
    ok = false;
    hipStream_t st = s->stream;
    Scalars *dsc = s->scal.as<Scalars>();
    Scalars hsc;
    // read groups of whole 64-read wave tiles, at most 2048 (k_refine2 run tables)
    const uint64_t ntiles = (nreads + 63) / 64;
    uint64_t gmax = RF_MAX_RUNS;
    uint64_t G = std::max<uint64_t>(1, std::min<uint64_t>(ntiles, gmax));
    const uint64_t gsize = ((ntiles + G - 1) / G) * 64;
    G = (nreads + gsize - 1) / gsize;
    auto npf_of = [](uint64_t lall) {  // 16-B chunks of a 64-read wave tile -> staged KiB per wave
        const uint64_t need16 = (64ull * lall + 30 + 15) / 16;
        return need16 <= 4 * 64 ? 4 : need16 <= 7 * 64 ? 7 : need16 <= 10 * 64 ? 10 : 0;
    };
    // super-k-mer fast path without the prescan (count_sk2.h, k_skpart_w<., ., true>): the
    // read length of the first read; the partition checks the rest
    if (allow_sk2 && k >= SK_MIN_K && k <= 32 && !kn().no_sk2) {
        uint64_t L = s->lc_L;  // (only a length the fast path then validates is reused)
        if (s->pipe.active) {
            L = s->pipe.first_len;  // host input: the host knows it
        } else if (!(L >= (uint64_t)k && npf_of(L) && s->lc_off == d_off && s->lc_n == nreads)) {
            uint64_t o2[2] = {0, 0};
            EC_CHECK(d2h(s, o2, d_off, 16, st));
            EC_CHECK(host_sync(s, st));
            L = o2[1] - o2[0];
        }
        s->lc_L = 0;  // cached again below only once the partition has validated it
        const int npf = npf_of(L);
        if (L >= (uint64_t)k && npf) {
            const uint32_t M = (uint32_t)(L - k + 1);
            bool done = false, invalid = false;
            mark(s, 2 * EC_STAGE_PRESCAN);  // (no prescan: the stage stays empty)
            mark(s, 2 * EC_STAGE_PRESCAN + 1);
            EC_CHECK(phase_count_sk2(s, d_reads, d_off, nreads, read_base, k, limit, M, G, gsize, nreads * M, npf, U,
                                     sidx, done, true, &invalid));
            if (done) {  // k_skpart_w<., ., true> checked every read against L
                if (!s->pipe.active) s->lc_off = d_off, s->lc_n = nreads, s->lc_L = L;
                ok = true;
                return EC_OK;
            }
            if (!invalid) allow_sk2 = false;  // the estimate or a capacity declined: window records
        }
    }
    EC_CHECK(pipe_all(s));
    mark(s, 2 * EC_STAGE_PRESCAN);
    kmark(s, 0, 0);
    k_prescan<<<(unsigned)G, 256, 0, st>>>(d_reads, d_off, nreads, k, gsize, &dsc->npos, &dsc->bad, dsc->lens);
    kmark(s, 0, 1);
    mark(s, 2 * EC_STAGE_PRESCAN + 1);
    EC_CHECK(d2h(s, &hsc, dsc, sizeof(Scalars), st));
    EC_CHECK(host_sync(s, st));
    if (hsc.bad != ~0ull) {
        uint8_t byte = 0;
        hipMemcpy(&byte, d_reads + hsc.bad, 1, hipMemcpyDeviceToHost);
        set_error("byte %llu (0x%02x) outside {A,C,G,T,N}", (unsigned long long)hsc.bad, byte);
        return EC_ERR_ALPHABET;
    }
    const unsigned int lmax = hsc.lens[0], lmin = ~hsc.lens[1], lall = hsc.lens[3];
    const uint64_t P = hsc.npos;
    if (hsc.lens[2] || P == 0 || lmax != lmin) return EC_OK;  // N, no windows, several lengths
    const uint32_t M = lmax - (uint32_t)k + 1;
    int ibits = 1;
    while ((1ull << ibits) < M) ibits++;
    if (ibits > 15 || nreads + read_base > (1ull << (31 - ibits)) || 2ull * M - 1 > MAX_LOCAL_EVENT) return EC_OK;
    const int npf = npf_of(lall);
    if (!npf) return EC_OK;
    if (allow_sk2) {  // super-k-mer records (count_sk2.h) unless window records are asked for
        bool done = false;
        EC_CHECK(phase_count_sk2(s, d_reads, d_off, nreads, read_base, k, limit, M, G, gsize, P, npf, U, sidx, done));
        if (done) {
            ok = true;
            return EC_OK;
        }
    }

    // 10-byte partition records (count_v2.h R10) where the hashed-key remnant and the
    // group-relative meta fit 80 bits (large inputs; EULERHIP_V2_R10 = 1 / 0 forces / disables)
    auto nbits = [](uint64_t x) {  // bits of the values 0 .. x - 1
        int b = 0;
        while ((1ull << b) < x) b++;
        return b;
    };
    const int r10env = kn().v2_r10;
    const bool r10 = r10env != 0 && (r10env == 1 || P >= (1ull << 26)) && k >= 16 &&
                     (2 * k - PT_CBITS) + std::max(0, nbits(gsize) + 1 + ibits - 16) <= 64;

    // ---- partition into fixed-capacity (coarse bucket, group) runs -------------------------
    constexpr uint64_t C = 1ull << PT_CBITS;
    const uint64_t cap = (gsize * M * 5 / 4 + C - 1) / C + 128;
    EC_CHECK(s->recs.ensure((C * G * cap + PT_REC) * 12));  // + the spill records
    EC_CHECK(s->cnt.ensure(C * G * 4));
    EC_CHECK(s->hll.ensure(G * (1 << HLL_REG_BITS)));
    EC_CHECK(s->ftot.ensure((1 << HLL_REG_BITS) * 4));
    unsigned long long *rkeys = s->recs.as<unsigned long long>();
    unsigned int *rmeta = reinterpret_cast<unsigned int *>(rkeys + C * G * cap + PT_REC);
    // HyperLogLog over a 1/256 sample of the key space on large inputs (~2 % error from 5·10^5
    // sampled keys up; the estimate only sizes the buckets)
    const uint32_t smask = P >= (1ull << 26) ? 255u : 0u;
    unsigned int *hreg = s->ftot.as<unsigned int>();
    mark(s, 2 * EC_STAGE_COUNT);
    kmark(s, 1, 0);
#define EC_PARTITION(NPF, HI, R10)                                                                            \
    k_partition<NPF, HI, R10><<<(unsigned)G, PT_THREADS, 0, st>>>(d_reads, d_off, nreads, k, M, gsize, (uint32_t)G, \
                                                                   cap, ibits, read_base, smask, rkeys, rmeta,        \
                                                                   s->cnt.as<unsigned int>(),                         \
                                                                   s->hll.as<uint8_t>(), &dsc->overflow)
#define EC_PARTITION_R(NPF, HI)        \
    if (r10)                           \
        EC_PARTITION(NPF, HI, true);   \
    else                               \
        EC_PARTITION(NPF, HI, false)
    if (k >= 17) {
        if (npf == 4) EC_PARTITION_R(4, true);
        else if (npf == 7) EC_PARTITION_R(7, true);
        else EC_PARTITION_R(10, true);
    } else {
        if (npf == 4) EC_PARTITION_R(4, false);
        else if (npf == 7) EC_PARTITION_R(7, false);
        else EC_PARTITION_R(10, false);
    }
#undef EC_PARTITION_R
#undef EC_PARTITION
    kmark(s, 1, 1);
    EC_HIP(hipMemsetAsync(hreg, 0, (1 << HLL_REG_BITS) * 4, st));
    k_hll_merge<<<dim3((1 << HLL_REG_BITS) / 256, TOT_SLICES), 256, 0, st>>>(s->hll.as<uint8_t>(), G, hreg);
    k_hll_final<<<1, 1024, 0, st>>>(hreg, HLL_REG_BITS, &dsc->est);
    EC_CHECK(d2h(s, &hsc, dsc, sizeof(Scalars), st));
    EC_CHECK(host_sync(s, st));
    if (hsc.overflow) return EC_OK;  // a run outgrew its capacity (extreme skew)
    const double est = hsc.est * (smask + 1.0);
    BucketPlan plan = plan_buckets(est, limit, !kn().no_filter);
    if (!plan.part) return EC_OK;
    plan.bbits = std::max(plan.bbits, PT_CBITS);
    const int bbits = plan.bbits;
    const uint64_t Bk = 1ull << bbits;

    // ---- refine into fixed-capacity final buckets -------------------------------------------
    const uint64_t fcap = P * 5 / 4 / Bk + 1024;
    EC_CHECK(s->recs2.ensure(Bk * fcap * 12));
    EC_CHECK(s->fcur.ensure(Bk * 8));
    EC_CHECK(s->bb2.ensure(Bk * 16));
    EC_HIP(hipMemsetAsync(s->fcur.p, 0, Bk * 8, st));
    unsigned rs = 8;
    if (kn().refine_rs) rs = (unsigned)std::max(1, kn().refine_rs);
    rs = (unsigned)std::min<uint64_t>(rs, G);
    kmark(s, 4, 0);
#define EC_REFINE(IN10)                                                                                           \
    k_refine2<IN10><<<dim3((unsigned)C, rs), BUCKET_THREADS, 0, st>>>(                                          \
        rkeys, rmeta, s->cnt.as<unsigned int>(), (uint32_t)G, cap, bbits, s->recs2.as<unsigned int>(), fcap,     \
        s->fcur.as<unsigned long long>(), &dsc->skew, k, ibits, gsize, read_base)
    if (r10)
        EC_REFINE(true);
    else
        EC_REFINE(false);
#undef EC_REFINE
    kmark(s, 4, 1);
    unsigned long long *bbeg = s->bb2.as<unsigned long long>(), *bend = bbeg + Bk;
    k_fixed_bounds<<<grid_for(Bk, 256), 256, 0, st>>>(s->fcur.as<unsigned long long>(), Bk, fcap, bbeg, bend);
    mark(s, 2 * EC_STAGE_COUNT + 1);

    // ---- count buckets in LDS tables ----------------------------------------------------------
    mark(s, 2 * EC_STAGE_COMPACT);
    const uint64_t umax = Bk * plan.slots;
    EC_CHECK(s->dkey.ensure(umax * 8));
    EC_CHECK(s->dcnt.ensure(umax * 4));
    EC_CHECK(s->dfc.ensure(umax * 8));
    EC_CHECK(s->dft.ensure(umax * 8));
    EC_CHECK(s->sub.ensure(umax * sizeof(SubSlot)));
    s->pmax = plan.pmax;
    s->part_keys = kn().part_keys > 0 ? kn().part_keys : (float)PART_KEYS;
    s->pmin = kn().filter_pmin >= 0 ? std::max(0, std::min(plan.pmax, kn().filter_pmin)) : 0;
    s->filt = plan.filt;
    s->bbeg = bbeg;
    s->bend = bend;
    kmark(s, 2, 0);
    const unsigned int m2 = 2 * M - 1;
    int rc;
    auto p12 = [&](auto &src) { src.ibits = ibits, src.k = k, src.m2 = m2, src.p = s->recs2.as<unsigned int>(); };
    if (r10 && (k & 1)) {  // the refine's key words hold h = bij_fwd(key)
        Rec12PSource<false, true> src;
        p12(src);
        rc = launch_bucket(s, src, (unsigned)Bk, plan.slots, limit);
    } else if (r10) {
        Rec12PSource<true, true> src;
        p12(src);
        rc = launch_bucket(s, src, (unsigned)Bk, plan.slots, limit);
    } else if (k & 1) {
        Rec12PSource<false> src;
        src.ibits = ibits, src.k = k, src.m2 = m2, src.p = s->recs2.as<unsigned int>();
        rc = launch_bucket(s, src, (unsigned)Bk, plan.slots, limit);
    } else {
        Rec12PSource<true> src;
        src.ibits = ibits, src.k = k, src.m2 = m2, src.p = s->recs2.as<unsigned int>();
        rc = launch_bucket(s, src, (unsigned)Bk, plan.slots, limit);
    }
    s->filt = false;
    s->bbeg = s->bend = nullptr;
    EC_CHECK(rc);
    kmark(s, 2, 1);
    mark(s, 2 * EC_STAGE_COMPACT + 1);
    EC_CHECK(d2h(s, &hsc, dsc, sizeof(Scalars), st));
    EC_CHECK(host_sync(s, st));
    if (hsc.overflow || hsc.skew) {  // a final bucket or an LDS table overflowed: redo on the exact path
        EC_HIP(hipMemsetAsync(dsc, 0, sizeof(Scalars), st));
        EC_HIP(hipMemsetAsync(&dsc->bad, 0xFF, sizeof(unsigned long long), st));
        s->stats.table_retries++;
        return EC_OK;
    }
    ok = true;
    s->stats.n_positions = P;
    s->stats.n_distinct_est = (uint64_t)llround(est);
    s->stats.record_bytes = r10 ? 10 : sizeof(Rec12);  // the partition's records (the refine writes 12 B)
    s->stats.n_records = P;
    s->stats.count_path = EC_PATH_PARTITIONED;
    s->stats.count_variant = r10 ? 2 : 1;
    s->stats.n_buckets = (uint32_t)Bk;
    s->stats.table_capacity = umax;
    sidx = SolidIndex{};
    sidx.sub = s->sub.as<SubSlot>();
    sidx.bbits = bbits;
    sidx.slots = plan.slots;
    sidx.sk = 0;
    sidx.npb = plan.filt ? s->bnp.as<uint8_t>() : nullptr;
    sidx.pmax = plan.pmax;
    sidx.bijk = r10 ? k : 0;  // R10 sub-tables hold bij_fwd(key)
    U = hsc.nsolid;
    s->stats.n_distinct = hsc.ndistinct;
    s->stats.n_solid = U;
    if (2ull * U >= (unsigned long long)CYC) {
        set_error("too many solid k-mers (%u) for 31-bit node ids", U);
        return EC_ERR_CAPACITY;
    }
    return EC_OK;
}

// build:25-42 on the device: count canonical k-mers of reads [0, nreads) (global read ids
// start at read_base), keep those with count > limit as dense arrays dkey/dcnt/dfc/dft (U of
// them) and a SolidIndex over them.
int phase_count(ec_session *s, const uint8_t *d_reads, const uint64_t *d_off, uint64_t nreads, uint64_t read_base,
                int k, long long limit, unsigned flags, unsigned int &U, SolidIndex &sidx) {
    if (nreads + read_base > (1ull << 32)) {
        set_error("global read ids reach %llu >= 2^32", (unsigned long long)(nreads + read_base));
        return EC_ERR_ARG;
    }
    s->stats.n_reads = nreads;
    hipStream_t st = s->stream;
    const unsigned B = 256;
    Scalars *dsc = s->scal.as<Scalars>();
    Scalars hsc;
    if (!(flags & (EC_FLAG_GENERAL | EC_FLAG_WIDE_RECORDS | EC_FLAG_EXACT_COUNT)) && nreads &&
        k <= 32 && !kn().no_v2) {
        bool ok = false;
        EC_CHECK(phase_count_v2(s, d_reads, d_off, nreads, read_base, k, limit, !(flags & EC_FLAG_WINDOW_RECORDS), U,
                                sidx, ok));
        if (ok) return EC_OK;
        EC_HIP(hipMemsetAsync(dsc, 0, sizeof(Scalars), st));
        EC_HIP(hipMemsetAsync(&dsc->bad, 0xFF, sizeof(unsigned long long), st));
    }
    EC_CHECK(pipe_all(s));

    // ---- prescan = partition upsweep ------------------------------------------------------
    mark(s, 2 * EC_STAGE_PRESCAN);
    const uint64_t ntiles = (nreads + TILE_READS - 1) / TILE_READS;
    uint64_t maxg = 2048;
    uint64_t ngroups = std::max<uint64_t>(1, std::min<uint64_t>(ntiles, maxg));
    const uint64_t gsize = std::max<uint64_t>(1, (ntiles + ngroups - 1) / ngroups) * TILE_READS;
    ngroups = std::max<uint64_t>(1, (nreads + gsize - 1) / gsize);
    EC_CHECK(s->hist.ensure(ngroups * FINE * 4));
    EC_CHECK(s->hll.ensure(ngroups * (1 << HLL_REG_BITS)));
    EC_CHECK(s->ftot.ensure((FINE + (1 << HLL_REG_BITS)) * 8));
    if (nreads) {
        kmark(s, 0, 0);
        k_upsweep<<<(unsigned)ngroups, TILE_READS, 0, st>>>(d_reads, d_off, nreads, k, gsize, s->hist.as<unsigned int>(),
                                                           s->hll.as<uint8_t>(), &dsc->npos, &dsc->bad, &dsc->maxlocal,
                                                           &dsc->skew, dsc->lens);
        kmark(s, 0, 1);
        EC_HIP(hipMemsetAsync(s->ftot.p, 0, (FINE + (1 << HLL_REG_BITS)) * 8, st));
        k_fine_totals<<<dim3(FINE / 256, TOT_SLICES), 256, 0, st>>>(
            s->hist.as<unsigned int>(), s->hll.as<uint8_t>(), ngroups, s->ftot.as<unsigned long long>(),
            reinterpret_cast<unsigned int *>(s->ftot.as<unsigned long long>() + FINE));
        k_hll_final<<<1, 1024, 0, st>>>(reinterpret_cast<unsigned int *>(s->ftot.as<unsigned long long>() + FINE),
                                        HLL_REG_BITS, &dsc->est);
    }
    mark(s, 2 * EC_STAGE_PRESCAN + 1);
    EC_CHECK(d2h(s, &hsc, dsc, sizeof(Scalars), st));
    EC_CHECK(host_sync(s, st));
    if (hsc.bad != ~0ull) {
        uint8_t byte = 0;
        hipMemcpy(&byte, d_reads + hsc.bad, 1, hipMemcpyDeviceToHost);
        set_error("byte %llu (0x%02x) outside {A,C,G,T,N}", (unsigned long long)hsc.bad, byte);
        return EC_ERR_ALPHABET;
    }
    const uint64_t P = nreads ? hsc.npos : 0;
    s->stats.n_positions = P;
    const double est = nreads ? hsc.est : 0.0;
    s->stats.n_distinct_est = (uint64_t)llround(est);

    // ---- count + compact ------------------------------------------------------------------
    // partitioned path when every bucket fits an LDS table and local events fit 16 bits
    // error-rich inputs (distinct keys >> solid keys) use the seen-twice filter buckets when a
    // key seen once cannot be solid by count alone (limit >= 1), up to ~32 K distinct per bucket
    // k_bucket_filt also splits a bucket into up to 2^PMAX part tables (large genomes; with
    // limit < 1 -- shard counts, no filter possible -- every key is kept)
    constexpr int PMAX = 3;
    const bool filt_ok = !kn().no_filter;
    const double filt_max = limit >= 1 ? 32768.0 : PART_KEYS * (1 << PMAX);
    bool part = !(flags & EC_FLAG_GENERAL) && nreads && P && hsc.maxlocal <= MAX_LOCAL_EVENT && !hsc.skew &&
                (est / FINE <= 2400.0 || (filt_ok && est / FINE <= filt_max));
    const bool filt = part && filt_ok && (est / FINE > 2400.0 || kn().force_filter);
    int pmax = 1;  // part tables per bucket region: 2^pmax (filter mode)
    while (pmax < PMAX && est / FINE / (double)(1 << pmax) > PART_KEYS) pmax++;
    if (kn().filter_pmax) pmax = std::max(1, std::min(PMAX, kn().filter_pmax));
    s->pmax = pmax;
    s->part_keys = kn().part_keys > 0 ? kn().part_keys : (float)PART_KEYS;
    s->pmin = kn().filter_pmin >= 0 ? std::max(0, std::min(pmax, kn().filter_pmin)) : 0;
    int bbits = 0;
    unsigned int slots = 2048;
    sidx = SolidIndex{};
    uint64_t umax = 0;
    if (part) {
        while (bbits < FINE_BITS && est / (double)(1ull << bbits) > 1100.0) bbits++;
        slots = filt ? (2048u << pmax) : est / (double)(1ull << bbits) > 1100.0 ? 4096u : 2048u;
        // fewest coarse buckets the refine fan-out allows: longer downsweep runs (measured:
        // 128 vs 256 coarse buckets, k_downsweep 5.56 -> 4.98 ms at 10M x 100 bp)
        int fan = 0;
        while ((1 << (fan + 1)) <= REFINE_FANOUT) fan++;
        int cbits = std::min(bbits, std::max(1, bbits - fan));
        const uint64_t Bk = 1ull << bbits, Ck = 1ull << cbits;
        mark(s, 2 * EC_STAGE_COUNT);
        EC_CHECK(s->cnt.ensure(Ck * ngroups * 8));
        EC_CHECK(s->offs.ensure(Ck * ngroups * 8));
        EC_CHECK(s->tot.ensure((Bk + 1) * 8));
        EC_CHECK(s->bstart.ensure((Bk + 1) * 8));
        // compact 12-B records: every read staged and N-free, one read length, events fit
        const unsigned int lmax = hsc.lens[0], lmin = ~hsc.lens[1];
        bool compact = !(flags & EC_FLAG_WIDE_RECORDS) && hsc.lens[2] == 0 && hsc.lens[1] != 0 && lmax == lmin;
        int ibits = 1;
        if (compact) {
            const uint64_t m = (uint64_t)lmax - (uint64_t)k + 1;
            while ((1ull << ibits) < m) ibits++;
            compact = ibits <= 15 && nreads + read_base <= (1ull << (31 - ibits));
        }
        const uint64_t NR = P;  // records
        const size_t rsz = compact ? sizeof(Rec12) : sizeof(Rec);
        s->stats.record_bytes = (uint32_t)rsz;
        s->stats.n_records = NR;
        EC_CHECK(s->recs.ensure(NR * rsz));
        if (bbits > cbits) EC_CHECK(s->recs2.ensure(NR * sizeof(Rec)));  // refine output
        k_coarse<<<grid_for(Ck * ngroups, B, 8192), B, 0, st>>>(s->hist.as<unsigned int>(), ngroups, cbits,
                                                               s->cnt.as<unsigned long long>());
        EC_CHECK(scan_u64(s, s->cnt.as<unsigned long long>(), s->offs.as<unsigned long long>(), Ck * ngroups));
        k_bucket_totals<<<grid_for(Bk + 1, B), B, 0, st>>>(s->ftot.as<unsigned long long>(), bbits,
                                                          s->tot.as<unsigned long long>());
        EC_CHECK(scan_u64(s, s->tot.as<unsigned long long>(), s->bstart.as<unsigned long long>(), Bk + 1));
        // compact records: keys [0, 8P) and meta [8P, 12P) of the first record buffer
        const Store12 c1{s->recs.as<unsigned long long>(), reinterpret_cast<unsigned int *>(s->recs.as<uint8_t>() + P * 8)};
        // refine output of compact records: packed 12-B records
        const bool pack12 = true;
        kmark(s, 1, 0);
        if (compact)
            k_downsweep<Rec12, MakeRec12, Store12><<<(unsigned)ngroups, TILE_READS, 0, st>>>(
                d_reads, d_off, nreads, k, gsize, ngroups, cbits, s->offs.as<unsigned long long>(), c1,
                MakeRec12{read_base, ibits});
        else
            k_downsweep<Rec, MakeRec, Store16><<<(unsigned)ngroups, TILE_READS, 0, st>>>(
                d_reads, d_off, nreads, k, gsize, ngroups, cbits, s->offs.as<unsigned long long>(),
                Store16{s->recs.as<Rec>()}, MakeRec{read_base});
        kmark(s, 1, 1);
        bool second = false;
        if (bbits > cbits) {
            // split every coarse bucket over RS workgroups (>= 4 per CU in flight)
            unsigned rsmax = 8;
            if (kn().refine_rs) rsmax = (unsigned)std::max(1, kn().refine_rs);
            const unsigned RS = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(rsmax, 1024 * rsmax / 8 / Ck));
            EC_CHECK(s->gcur.ensure(Bk * 8));
            EC_HIP(hipMemcpyAsync(s->gcur.p, s->bstart.p, Bk * 8, hipMemcpyDeviceToDevice, st));
            kmark(s, 4, 0);
            if (compact && pack12)  // 12-B in, packed 12-B out
                k_refine<Rec12, Store12, Store12P><<<dim3((unsigned)Ck, RS), BUCKET_THREADS, 0, st>>>(
                    c1, Store12P{s->recs2.as<unsigned int>()}, s->bstart.as<unsigned long long>(),
                    s->gcur.as<unsigned long long>(), cbits, bbits);
            else if (compact)  // 12-B in, 16-B out: k_bucket reads 16-B records
                k_refine<Rec12, Store12, Store12to16><<<dim3((unsigned)Ck, RS), BUCKET_THREADS, 0, st>>>(
                    c1, Store12to16{s->recs2.as<Rec>(), ibits, k, (unsigned int)(2 * ((uint64_t)lmax - k + 1) - 1)},
                    s->bstart.as<unsigned long long>(), s->gcur.as<unsigned long long>(), cbits, bbits);
            else
                k_refine<Rec, Store16, Store16><<<dim3((unsigned)Ck, RS), BUCKET_THREADS, 0, st>>>(
                    Store16{s->recs.as<Rec>()}, Store16{s->recs2.as<Rec>()}, s->bstart.as<unsigned long long>(),
                    s->gcur.as<unsigned long long>(), cbits, bbits);
            kmark(s, 4, 1);
            second = true;
        }
        mark(s, 2 * EC_STAGE_COUNT + 1);
        mark(s, 2 * EC_STAGE_COMPACT);
        umax = Bk * slots;
        EC_CHECK(s->dkey.ensure(umax * 8));
        EC_CHECK(s->dcnt.ensure(umax * 4));
        EC_CHECK(s->dfc.ensure(umax * 8));
        EC_CHECK(s->dft.ensure(umax * 8));
        EC_CHECK(s->sub.ensure(umax * sizeof(SubSlot)));
        kmark(s, 2, 0);
        s->filt = filt;
        if (compact && second && pack12) {
            const unsigned int m2 = (unsigned int)(2 * ((uint64_t)lmax - k + 1) - 1);
            if (k & 1) {
                Rec12PSource<false> src;
                src.ibits = ibits, src.k = k, src.m2 = m2, src.p = s->recs2.as<unsigned int>();
                EC_CHECK(launch_bucket(s, src, (unsigned)Bk, slots, (long long)limit));
            } else {
                Rec12PSource<true> src;
                src.ibits = ibits, src.k = k, src.m2 = m2, src.p = s->recs2.as<unsigned int>();
                EC_CHECK(launch_bucket(s, src, (unsigned)Bk, slots, (long long)limit));
            }
        } else if (compact && !second) {
            const unsigned int m2 = (unsigned int)(2 * ((uint64_t)lmax - k + 1) - 1);
            if (k & 1) {
                Rec12Source<false> src;
                src.ibits = ibits, src.k = k, src.m2 = m2, src.key = c1.key, src.meta = c1.meta;
                EC_CHECK(launch_bucket(s, src, (unsigned)Bk, slots, (long long)limit));
            } else {
                Rec12Source<true> src;
                src.ibits = ibits, src.k = k, src.m2 = m2, src.key = c1.key, src.meta = c1.meta;
                EC_CHECK(launch_bucket(s, src, (unsigned)Bk, slots, (long long)limit));
            }
        } else {
            EC_CHECK(launch_bucket(s, RecSource{second ? s->recs2.as<Rec>() : s->recs.as<Rec>()}, (unsigned)Bk, slots,
                                   (long long)limit));
        }
        s->filt = false;
        kmark(s, 2, 1);
        mark(s, 2 * EC_STAGE_COMPACT + 1);
        EC_CHECK(d2h(s, &hsc, dsc, sizeof(Scalars), st));
        EC_CHECK(host_sync(s, st));
        if (hsc.overflow) {  // a bucket outgrew its LDS table: redo on the general path
            part = false;
            s->stats.table_retries++;
            EC_HIP(hipMemsetAsync(&dsc->nsolid, 0, 4, st));
            EC_HIP(hipMemsetAsync(&dsc->ndistinct, 0, 8, st));
            EC_HIP(hipMemsetAsync(&dsc->overflow, 0, 4, st));
        } else {
            sidx.sub = s->sub.as<SubSlot>();
            sidx.bbits = bbits;
            sidx.slots = slots;
            sidx.sk = 0;
            sidx.npb = filt ? s->bnp.as<uint8_t>() : nullptr;
            sidx.pmax = pmax;
            s->stats.count_path = EC_PATH_PARTITIONED;
            s->stats.n_buckets = (uint32_t)Bk;
            s->stats.table_capacity = umax;
        }
    }
    if (!part) {
        uint64_t want = (uint64_t)(std::max<double>(est, 1.0) * 2.2) + 1024;
        want = std::min<uint64_t>(want, 2 * P + 1024);
        uint64_t cap = 1024;
        while (cap < want) cap <<= 1;
        for (int attempt = 0;; attempt++) {
            EC_CHECK(s->table.ensure(cap * sizeof(Slot)));
            mark(s, 2 * EC_STAGE_COUNT);
            k_table_clear<<<grid_for(cap, B, 8192), B, 0, st>>>(s->table.as<Slot>(), cap);
            EC_HIP(hipMemsetAsync(&dsc->overflow, 0, 4, st));
            kmark(s, 3, 0);
            if (nreads)
                k_count<<<grid_for(nreads, B), B, 0, st>>>(d_reads, d_off, nreads, k, s->table.as<Slot>(), cap - 1,
                                                          &dsc->overflow, read_base);
            kmark(s, 3, 1);
            mark(s, 2 * EC_STAGE_COUNT + 1);
            EC_CHECK(d2h(s, &hsc.overflow, &dsc->overflow, 4, st));
            EC_CHECK(host_sync(s, st));
            if (!hsc.overflow) break;
            if (attempt >= 4) {
                set_error("hash table overflow at capacity %llu", (unsigned long long)cap);
                return EC_ERR_CAPACITY;
            }
            cap <<= 2;
            s->stats.table_retries++;
        }
        s->stats.table_capacity = cap;
        mark(s, 2 * EC_STAGE_COMPACT);
        umax = cap;
        EC_CHECK(s->dkey.ensure(umax * 8));
        EC_CHECK(s->dcnt.ensure(umax * 4));
        EC_CHECK(s->dfc.ensure(umax * 8));
        EC_CHECK(s->dft.ensure(umax * 8));
        EC_CHECK(compact_table(s, s->table.as<Slot>(), cap, (long long)limit, s->dkey.as<unsigned long long>()));
        mark(s, 2 * EC_STAGE_COMPACT + 1);
        EC_CHECK(d2h(s, &hsc, dsc, sizeof(Scalars), st));
        EC_CHECK(host_sync(s, st));
        sidx.table = s->table.as<Slot>();
        sidx.capmask = cap - 1;
        s->stats.count_path = EC_PATH_GENERAL;
    }
    U = hsc.nsolid;
    s->stats.n_distinct = hsc.ndistinct;
    s->stats.n_solid = U;
    if (2ull * U >= (unsigned long long)CYC) {
        set_error("too many solid k-mers (%u) for 31-bit node ids", U);
        return EC_ERR_CAPACITY;
    }
    return EC_OK;
}

// Owner-side aggregation of exchanged k-mer records (count sum, first-event min) followed by
// the solid filter: the merge step of the sharded path, and the way a gathered solid set is
// loaded for phase_graph (limit = keep all).
// The same on the LDS bucket tables of the fused path (k_bucket over the records sorted by
// bucket): no HBM atomics.  Returns EC_OK with ok = false when a bucket overflows its table.
// minimizer buckets for the merge / load of 21 <= k <= 32 (shard.h OwnerFn; EULERHIP_MERGE_MIX=1:
// key-hash buckets and owners, the round-1 layout)
bool merge_sk(int k) { return k >= SK_MIN_K && k <= 32 && !kn().merge_mix; }
// 128-bit keys on minimizer owners (the count's minimizer buckets, count_wide.h)
bool merge_wmb(int k) { return k > 32 && k <= WMB_MAX_K && kn().wide_mb != 0 && !kn().merge_mix; }
OwnerFn owner_fn(int k) {
    OwnerFn f{};
    f.sk = merge_sk(k) ? 1 : 0;
    if (f.sk) f.mc = sk_cfg(k);
    f.wk = merge_wmb(k) ? k : 0;
    return f;
}

// counting sort of n > 0 bin ids (shard.h k_cs_*): perm in midx2, bin starts bstart[0..nbins)
// (end: and bstart[nbins] = n)
int cs_sort(ec_session *s, const unsigned int *bid, uint64_t n, unsigned int nbins, unsigned long long *bstart,
            bool end = false) {
    hipStream_t st = s->stream;
    const unsigned int nch = (unsigned int)((n + CS_CHUNK - 1) / CS_CHUNK);
    EC_CHECK(s->midx2.ensure(std::max<uint64_t>(n, 1) * 4));
    EC_CHECK(s->mbid2.ensure(std::max<uint64_t>(n, 3ull * nbins) * 4));  // (mbid2 is free here)
    unsigned int *tot = s->mbid2.as<unsigned int>(), *incl = tot + nbins, *cur = incl + nbins;
    EC_HIP(hipMemsetAsync(tot, 0, (size_t)nbins * 4, st));
    k_cs_hist<<<nch, 1024, nbins * 4, st>>>(bid, n, nbins, tot);
    EC_CHECK(scan_incl_u32(s, tot, incl, nbins));
    k_cs_starts<<<grid_for(nbins, 256), 256, 0, st>>>(tot, incl, nbins, bstart, cur, end);
    k_cs_scatter<<<nch, 1024, nbins * 4, st>>>(bid, n, nbins, cur, s->midx2.as<unsigned int>());
    return EC_OK;
}

int phase_merge_part(ec_session *s, const Agg *d_agg, uint64_t n, long long limit, unsigned int &U, SolidIndex &sidx,
                     bool &ok, const unsigned int *ids = nullptr, bool allow_sk = true, const XIn *xin = nullptr) {
    // (xin: the received records read in place, ec_merge_owned_from; d_agg unused)
    hipStream_t st = s->stream;
    const unsigned B = 256;
    Scalars *dsc = s->scal.as<Scalars>();
    Scalars hsc;
    ok = false;
    int bbits = 0;
    while (bbits < FINE_BITS && (double)n / (double)(1ull << bbits) > 1100.0) bbits++;
    if ((double)n / (double)(1ull << bbits) > 2200.0) return EC_OK;  // too large for the LDS tables
    const unsigned int nb = 1u << bbits;
    const unsigned int slots = (double)n / (double)nb > 1100.0 ? 4096u : 2048u;
    OwnerFn own = owner_fn(s->k);  // minimizer buckets (own.sk) or key-hash buckets
    if (!allow_sk) own.sk = 0;
    mark(s, 2 * EC_STAGE_COUNT);
    EC_CHECK(s->mbid.ensure(std::max<uint64_t>(n, 1) * 4));
    EC_CHECK(s->mbid2.ensure(std::max<uint64_t>(n, 1) * 4));
    EC_CHECK(s->midx2.ensure(std::max<uint64_t>(n, 1) * 4));
    EC_CHECK(s->bstart.ensure((nb + 1ull) * 8));
    if (!n) EC_HIP(hipMemsetAsync(s->bstart.p, 0, (nb + 1ull) * 8, st));  // (else k_cs_starts writes them all)
    if (n) {
        if (xin)
            k_agg_bucket_ids<XIn><<<grid_for(n, B), B, 0, st>>>(*xin, n, bbits, s->mbid.as<unsigned int>(), own.mc,
                                                               own.sk);
        else
            k_agg_bucket_ids<PlainIn><<<grid_for(n, B), B, 0, st>>>(PlainIn{d_agg}, n, bbits, s->mbid.as<unsigned int>(),
                                                                   own.mc, own.sk);
        // indices by bucket: counting sort (shard.h k_cs_*), buckets 0..nb (nb: filler records)
        EC_CHECK(cs_sort(s, s->mbid.as<unsigned int>(), n, nb + 1, s->bstart.as<unsigned long long>()));
    }
    mark(s, 2 * EC_STAGE_COUNT + 1);
    mark(s, 2 * EC_STAGE_COMPACT);
    const uint64_t umax = (uint64_t)nb * slots;
    EC_CHECK(s->dkey.ensure(umax * 8));
    EC_CHECK(s->dcnt.ensure(umax * 4));
    EC_CHECK(s->dfc.ensure(umax * 8));
    EC_CHECK(s->dft.ensure(umax * 8));
    EC_CHECK(s->sub.ensure(umax * sizeof(SubSlot)));
    // ndistinct, est, overflow, nsolid: one fill (they are adjacent; est is the count's alone)
    static_assert(offsetof(Scalars, nsolid) + 4 - offsetof(Scalars, ndistinct) == 24, "Scalars layout");
    EC_HIP(hipMemsetAsync(&dsc->ndistinct, 0, 24, st));
    kmark(s, 2, 0);
    const int sks = own.sk ? (slots == 2048 ? 11 : 12) : 0;
    bool merge_marked = false;
    if (!ids) s->seg_marks = 0;
    if (ids) {  // gathered solid set: dense ids given (partitioned graph phase)
        const AggDetSource src{d_agg, s->midx2.as<unsigned int>(), ids, sks};
        EC_CHECK(launch_bucket(s, src, nb, slots, limit));
    } else {
        // (minimizer buckets: their first ids marked for the partitioned finish's tiles)
        unsigned int *bm = nullptr;
        if (own.sk && !s->filt && kn().tile_plan != 0) {
            const size_t words = umax / 32 + 2;
            EC_CHECK(s->bmark.ensure(words * 4));
            EC_HIP(hipMemsetAsync(s->bmark.p, 0, words * 4, st));
            bm = s->bmark.as<unsigned int>();
        }
        if (xin) {
            const XAggSource src{*xin, s->midx2.as<unsigned int>(), sks};
            EC_CHECK(launch_bucket(s, src, nb, slots, limit, bm));
        } else {
            const AggSource src{d_agg, s->midx2.as<unsigned int>(), sks};
            EC_CHECK(launch_bucket(s, src, nb, slots, limit, bm));
        }
        merge_marked = bm != nullptr;
    }
    kmark(s, 2, 1);
    mark(s, 2 * EC_STAGE_COMPACT + 1);
    EC_CHECK(d2h(s, &hsc, dsc, sizeof(Scalars), st));
    EC_CHECK(host_sync(s, st));
    if (hsc.overflow) {
        s->stats.table_retries++;
        EC_HIP(hipMemsetAsync(&dsc->overflow, 0, 4, st));
        return EC_OK;
    }
    U = ids ? hsc.ngath : hsc.nsolid;  // ids: the dense ids k_det_ids gave (their count in ngath)
    s->stats.n_distinct = U;
    if (!ids) s->stats.n_distinct = hsc.ndistinct;
    s->stats.n_solid = U;
    s->stats.count_path = EC_PATH_PARTITIONED;
    s->stats.n_buckets = nb;
    s->stats.table_capacity = umax;
    sidx = SolidIndex{};
    sidx.sub = s->sub.as<SubSlot>();
    sidx.bbits = bbits;
    sidx.slots = slots;
    sidx.sk = own.sk;
    if (own.sk) sidx.mc = own.mc;
    if (2ull * U >= (unsigned long long)CYC) {
        set_error("too many solid k-mers (%u) for 31-bit node ids", U);
        return EC_ERR_CAPACITY;
    }
    if (merge_marked) s->seg_marks = U;  // (bmark holds this merge's bucket starts, U ids)
    ok = true;
    return EC_OK;
}

int phase_merge(ec_session *s, const Agg *d_agg, uint64_t n, long long limit, unsigned int &U, SolidIndex &sidx,
                const XIn *xin = nullptr, const std::function<int(const Agg *&)> &decode = nullptr) {
    if (!(s->flags & EC_FLAG_GENERAL)) {
        bool ok = false;
        EC_CHECK(phase_merge_part(s, d_agg, n, limit, U, sidx, ok, nullptr, true, xin));
        if (!ok && merge_sk(s->k)) EC_CHECK(phase_merge_part(s, d_agg, n, limit, U, sidx, ok, nullptr, false, xin));
        if (ok) return EC_OK;
    }
    if (xin) EC_CHECK(decode(d_agg));  // the HBM table reads decoded records
    hipStream_t st = s->stream;
    const unsigned B = 256;
    Scalars *dsc = s->scal.as<Scalars>();
    Scalars hsc;
    uint64_t cap = 1024;
    while (cap < (uint64_t)(2.2 * (double)n) + 1024) cap <<= 1;
    for (int attempt = 0;; attempt++) {
        EC_CHECK(s->table.ensure(cap * sizeof(Slot)));
        mark(s, 2 * EC_STAGE_COUNT);
        k_table_clear<<<grid_for(cap, B, 8192), B, 0, st>>>(s->table.as<Slot>(), cap);
        EC_HIP(hipMemsetAsync(&dsc->overflow, 0, 4, st));
        if (n) k_merge_agg<<<grid_for(n, B), B, 0, st>>>(d_agg, n, s->table.as<Slot>(), cap - 1, &dsc->overflow);
        mark(s, 2 * EC_STAGE_COUNT + 1);
        EC_CHECK(d2h(s, &hsc.overflow, &dsc->overflow, 4, st));
        EC_CHECK(host_sync(s, st));
        if (!hsc.overflow) break;
        if (attempt >= 4) {
            set_error("merge table overflow at capacity %llu", (unsigned long long)cap);
            return EC_ERR_CAPACITY;
        }
        cap <<= 2;
        s->stats.table_retries++;
    }
    s->stats.table_capacity = cap;
    mark(s, 2 * EC_STAGE_COMPACT);
    EC_CHECK(s->dkey.ensure(cap * 8));
    EC_CHECK(s->dcnt.ensure(cap * 4));
    EC_CHECK(s->dfc.ensure(cap * 8));
    EC_CHECK(s->dft.ensure(cap * 8));
    EC_HIP(hipMemsetAsync(&dsc->nsolid, 0, 4, st));
    EC_HIP(hipMemsetAsync(&dsc->ndistinct, 0, 8, st));
    EC_CHECK(compact_table(s, s->table.as<Slot>(), cap, limit, s->dkey.as<unsigned long long>()));
    mark(s, 2 * EC_STAGE_COMPACT + 1);
    EC_CHECK(d2h(s, &hsc, dsc, sizeof(Scalars), st));
    EC_CHECK(host_sync(s, st));
    U = hsc.nsolid;
    s->stats.n_distinct = hsc.ndistinct;
    s->stats.n_solid = U;
    s->stats.count_path = EC_PATH_GENERAL;
    sidx = SolidIndex{};
    sidx.table = s->table.as<Slot>();
    sidx.capmask = cap - 1;
    if (2ull * U >= (unsigned long long)CYC) {
        set_error("too many solid k-mers (%u) for 31-bit node ids", U);
        return EC_ERR_CAPACITY;
    }
    return EC_OK;
}


// partitioned graph phase: the all-gathered solid set with dense ids = position among the
// non-filler records (owner-major), identical on every rank, plus the bucketed lookup index
int phase_load_det(ec_session *s, const Agg *d_agg, uint64_t n, unsigned int &U, SolidIndex &sidx) {
    hipStream_t st = s->stream;
    Scalars *dsc = s->scal.as<Scalars>();
    const unsigned int nblk = (unsigned int)std::max<uint64_t>((n + DET_CHUNK - 1) / DET_CHUNK, 1);
    EC_CHECK(s->rbc.ensure((size_t)nblk * 8));
    EC_CHECK(s->nextR.ensure(std::max<uint64_t>(n, 1) * 4));  // ids (nextR is free until the rank stage)
    unsigned int *bc = s->rbc.as<unsigned int>(), *bs = bc + nblk, *ids = s->nextR.as<unsigned int>();
    // the id count stays on the device (dsc->ngath, read back with phase_merge_part's scalars):
    // the dense arrays are sized for all n records, so no host round trip here
    EC_HIP(hipMemsetAsync(&dsc->ngath, 0, 4, st));
    if (n) {
        k_det_count<Agg><<<nblk, 256, 0, st>>>(d_agg, n, bc);
        EC_CHECK(scan_incl_u32(s, bc, bs, nblk));
        k_det_ids<Agg><<<nblk, 256, 0, st>>>(d_agg, n, bs, ids);
        EC_HIP(hipMemcpyAsync(&dsc->ngath, bs + nblk - 1, 4, hipMemcpyDeviceToDevice, st));
    }
    EC_CHECK(s->dkey.ensure(std::max<uint64_t>(n, 1) * 8));
    EC_CHECK(s->dcnt.ensure(std::max<uint64_t>(n, 1) * 4));
    EC_CHECK(s->dfc.ensure(std::max<uint64_t>(n, 1) * 8));
    EC_CHECK(s->dft.ensure(std::max<uint64_t>(n, 1) * 8));
    bool ok = false;
    EC_CHECK(phase_merge_part(s, d_agg, n, LLONG_MIN, U, sidx, ok, ids));
    // a minimizer bucket past its table (low-complexity sequence: many keys, one minimizer):
    // key-hash buckets instead
    if (!ok && merge_sk(s->k)) EC_CHECK(phase_merge_part(s, d_agg, n, LLONG_MIN, U, sidx, ok, ids, false));
    if (!ok) {
        set_error("gathered solid set of %llu records does not fit the bucketed index", (unsigned long long)n);
        return EC_ERR_CAPACITY;
    }
    (void)dsc;
    return EC_OK;
}

// the same for k > 32: dense arrays in gathered order, HBM lookup table (SolidIndexW)
int phase_load_det_w(ec_session *s, const AggW *d_agg, uint64_t n, unsigned int &U, SolidIndexW &sidx) {
    hipStream_t st = s->stream;
    const unsigned B = 256;
    Scalars *dsc = s->scal.as<Scalars>();
    const unsigned int nblk = (unsigned int)std::max<uint64_t>((n + DET_CHUNK - 1) / DET_CHUNK, 1);
    EC_CHECK(s->rbc.ensure((size_t)nblk * 8));
    EC_CHECK(s->nextR.ensure(std::max<uint64_t>(n, 1) * 4));
    unsigned int *bc = s->rbc.as<unsigned int>(), *bs = bc + nblk, *ids = s->nextR.as<unsigned int>();
    unsigned int tot = 0;
    if (n) {
        k_det_count<AggW><<<nblk, 256, 0, st>>>(d_agg, n, bc);
        EC_CHECK(scan_incl_u32(s, bc, bs, nblk));
        k_det_ids<AggW><<<nblk, 256, 0, st>>>(d_agg, n, bs, ids);
        EC_CHECK(d2h(s, &tot, bs + nblk - 1, 4, st));
        EC_CHECK(host_sync(s, st));
    }
    EC_CHECK(s->dkey.ensure(std::max<uint64_t>(tot, 1) * sizeof(K128)));
    EC_CHECK(s->dcnt.ensure(std::max<uint64_t>(tot, 1) * 4));
    EC_CHECK(s->dfc.ensure(std::max<uint64_t>(tot, 1) * 8));
    EC_CHECK(s->dft.ensure(std::max<uint64_t>(tot, 1) * 8));
    uint64_t cap = 1024;
    while (cap < (uint64_t)(2.2 * (double)tot) + 1024) cap <<= 1;
    for (int attempt = 0;; attempt++) {
        EC_CHECK(s->table.ensure(cap * sizeof(SlotW)));
        mark(s, 2 * EC_STAGE_COUNT);
        k_table_clear_w<<<grid_for(cap, B, 8192), B, 0, st>>>(s->table.as<SlotW>(), cap);
        EC_HIP(hipMemsetAsync(&dsc->overflow, 0, 4, st));
        if (n)
            k_load_det_w<<<grid_for(n, B), B, 0, st>>>(d_agg, n, ids, s->table.as<SlotW>(), cap - 1, s->dkey.as<K128>(),
                                                      s->dcnt.as<unsigned int>(), s->dfc.as<unsigned long long>(),
                                                      s->dft.as<unsigned long long>(), &dsc->overflow);
        mark(s, 2 * EC_STAGE_COUNT + 1);
        unsigned int of = 0;
        EC_CHECK(d2h(s, &of, &dsc->overflow, 4, st));
        EC_CHECK(host_sync(s, st));
        if (!of) break;
        if (attempt >= 4) {
            set_error("load table overflow at capacity %llu", (unsigned long long)cap);
            return EC_ERR_CAPACITY;
        }
        cap <<= 2;
        s->stats.table_retries++;
    }
    U = tot;
    s->stats.n_distinct = tot;
    s->stats.n_solid = tot;
    s->stats.table_capacity = cap;
    sidx.table = s->table.as<SlotW>();
    sidx.capmask = cap - 1;
    sidx.sub = nullptr;
    return EC_OK;
}

// ---- 32 < k <= 63: 128-bit keys (wide.h), general-table counting ---------------------------
int finish_wide(ec_session *s, uint64_t cap, long long limit, unsigned int &U, SolidIndexW &sidx,
                uint64_t ubound = 0) {
    hipStream_t st = s->stream;
    Scalars *dsc = s->scal.as<Scalars>();
    Scalars hsc;
    mark(s, 2 * EC_STAGE_COMPACT);
    // (ubound: at most that many keys -- a merge's records; the table's capacity otherwise)
    const uint64_t ucap = ubound ? std::min<uint64_t>(cap, ubound) : cap;
    EC_CHECK(s->dkey.ensure(std::max<uint64_t>(ucap, 1) * sizeof(K128)));
    EC_CHECK(s->dcnt.ensure(std::max<uint64_t>(ucap, 1) * 4));
    EC_CHECK(s->dfc.ensure(std::max<uint64_t>(ucap, 1) * 8));
    EC_CHECK(s->dft.ensure(std::max<uint64_t>(ucap, 1) * 8));
    EC_HIP(hipMemsetAsync(&dsc->nsolid, 0, 4, st));
    EC_HIP(hipMemsetAsync(&dsc->ndistinct, 0, 8, st));
    EC_CHECK(compact_table(s, s->table.as<SlotW>(), cap, limit, s->dkey.as<K128>()));
    mark(s, 2 * EC_STAGE_COMPACT + 1);
    EC_CHECK(d2h(s, &hsc, dsc, sizeof(Scalars), st));
    EC_CHECK(host_sync(s, st));
    U = hsc.nsolid;
    s->stats.n_distinct = hsc.ndistinct;
    s->stats.n_solid = U;
    s->stats.count_path = EC_PATH_GENERAL;
    s->stats.table_capacity = cap;
    sidx.table = s->table.as<SlotW>();
    sidx.capmask = cap - 1;
    sidx.sub = nullptr;
    if (2ull * U >= (unsigned long long)CYC) {
        set_error("too many solid k-mers (%u) for 31-bit node ids", U);
        return EC_ERR_CAPACITY;
    }
    return EC_OK;
}

// Partitioned wide count (count_wide.h): upsweep, downsweep, refine and one LDS table per
// bucket, as phase_count for k <= 32.  ok = false (scalars reset) when the input needs the
// HBM table: reads with 'N' or other bytes, tiles over the 40 KB stage, a bucket past its table.
int phase_count_wpart(ec_session *s, const uint8_t *d_reads, const uint64_t *d_off, uint64_t nreads,
                      uint64_t read_base, int k, long long limit, unsigned int &U, SolidIndexW &sidx, bool &ok,
                      bool mb = false, bool *mb_declined = nullptr) {
    ok = false;
    if ((s->flags & EC_FLAG_GENERAL) || !nreads || kn().wide_general) return EC_OK;
    hipStream_t st = s->stream;
    const unsigned B = 256;
    Scalars *dsc = s->scal.as<Scalars>();
    Scalars hsc;
    auto reset = [&]() -> int {
        EC_HIP(hipMemsetAsync(dsc, 0, sizeof(Scalars), st));
        EC_HIP(hipMemsetAsync(&dsc->bad, 0xFF, sizeof(unsigned long long), st));
        return EC_OK;
    };
    mark(s, 2 * EC_STAGE_PRESCAN);
    const uint64_t ntiles = (nreads + TILE_READS - 1) / TILE_READS;
    uint64_t maxg = 2048;
    uint64_t ngroups = std::max<uint64_t>(1, std::min<uint64_t>(ntiles, maxg));
    const uint64_t gsize = std::max<uint64_t>(1, (ntiles + ngroups - 1) / ngroups) * TILE_READS;
    ngroups = std::max<uint64_t>(1, (nreads + gsize - 1) / gsize);
    constexpr int HR = 1 << HLL_REG_BITS;
    EC_CHECK(s->hist.ensure(ngroups * FINE_W * 4));
    EC_CHECK(s->hll.ensure(ngroups * HR));
    EC_CHECK(s->ftot.ensure((FINE_W + HR) * 8));
    kmark(s, 0, 0);
    // minimizer buckets (count_wide.h k_wbv): every window's minimizer, indexed by its base offset
    uint32_t *wbv = nullptr;
    uint32_t mbM = 0;
    uint32_t *rpack = nullptr, rpack_d = 0;
    if (mb) {  // reads of one length L <= WMB_MAXL only (k_wbv checks the others)
        uint64_t o2[2] = {0, 0};
        EC_CHECK(d2h(s, o2, d_off, 16, st));
        EC_CHECK(host_sync(s, st));
        const uint64_t L = o2[1] - o2[0];
        if (L < (uint64_t)k || L > WMB_MAXL) {
            if (mb_declined) *mb_declined = true;
            return reset();
        }
        mbM = (uint32_t)(L - k + 1);
        EC_HIP(hipMemsetAsync(&dsc->wbv_long, 0, 4, st));
        EC_CHECK(s->wbv.ensure(((nreads + 255) / 256) * 256 * (uint64_t)mbM * 4));
        wbv = s->wbv.as<uint32_t>();
        const unsigned g = (unsigned)((nreads + 63) / 64);
        // large inputs (the third level's run codes): k_wbv also writes the reads as 2-bit codes,
        // from which k_run_codes copies each run's codes (EULERHIP_RUN_PACKED=0: from the ASCII)
        if (kn().wide_runs != 0 && kn().run_packed != 0 && (uint64_t)nreads * mbM >= (1ull << 26)) {
            rpack_d = (uint32_t)((L + 15) / 16);
            EC_CHECK(s->rpack.ensure((uint64_t)nreads * rpack_d * 4));
            rpack = s->rpack.as<uint32_t>();
        }
        switch (k - SK_M + 1) {  // (WMB_MAX_K = 52: w <= 38)
#define EC_WBV(W) \
    case W: k_wbv<W><<<g, 64, 0, st>>>(d_reads, d_off, nreads, (uint32_t)L, wbv, &dsc->wbv_long, rpack, rpack_d); break;
            EC_WBV(19) EC_WBV(20) EC_WBV(21) EC_WBV(22) EC_WBV(23) EC_WBV(24) EC_WBV(25) EC_WBV(26) EC_WBV(27)
            EC_WBV(28) EC_WBV(29) EC_WBV(30) EC_WBV(31) EC_WBV(32) EC_WBV(33) EC_WBV(34) EC_WBV(35) EC_WBV(36)
            EC_WBV(37) EC_WBV(38)
#undef EC_WBV
            default: set_error("minimizer buckets: k = %d out of range", k); return EC_ERR_ARG;
        }
    }
    // minimizer runs as the partition records (count_wide.h RunWM; EULERHIP_WIDE_RUNS=0: windows)
    const bool runs = mb && kn().wide_runs != 0;
    // HyperLogLog sampled by minimizer past ~6.7e7 positions (as the super-k-mer count)
    const uint32_t hsmask = mb && (uint64_t)nreads * mbM >= (1ull << 26) ? 255u : 0u;
    if (runs && kn().upsweep_staged != 1)
        k_upsweep_runs<<<(unsigned)ngroups, TILE_READS, 0, st>>>(d_reads, d_off, nreads, k, gsize,
                                                                s->hist.as<unsigned int>(), s->hll.as<uint8_t>(),
                                                                &dsc->npos, &dsc->maxlocal, &dsc->skew, wbv, mbM,
                                                                hsmask);
    else if (runs)  // (EULERHIP_UPSWEEP_STAGED=1: the staged kernel, A/B)
        k_upsweep_w<true, true><<<(unsigned)ngroups, TILE_READS, 0, st>>>(d_reads, d_off, nreads, k, gsize,
                                                                         s->hist.as<unsigned int>(), s->hll.as<uint8_t>(),
                                                                         &dsc->npos, &dsc->maxlocal, &dsc->skew,
                                                                         dsc->lens, wbv, mbM, hsmask);
    else if (mb)
        k_upsweep_w<true><<<(unsigned)ngroups, TILE_READS, 0, st>>>(d_reads, d_off, nreads, k, gsize,
                                                                   s->hist.as<unsigned int>(), s->hll.as<uint8_t>(),
                                                                   &dsc->npos, &dsc->maxlocal, &dsc->skew, dsc->lens,
                                                                   wbv, mbM, hsmask);
    else
        k_upsweep_w<false><<<(unsigned)ngroups, TILE_READS, 0, st>>>(d_reads, d_off, nreads, k, gsize,
                                                                    s->hist.as<unsigned int>(), s->hll.as<uint8_t>(),
                                                                    &dsc->npos, &dsc->maxlocal, &dsc->skew, dsc->lens,
                                                                    nullptr, 0u);
    kmark(s, 0, 1);
    unsigned long long *ftot = s->ftot.as<unsigned long long>();
    EC_HIP(hipMemsetAsync(ftot, 0, (FINE_W + HR) * 8, st));
    EC_HIP(hipMemsetAsync(&dsc->nrec, 0, sizeof(unsigned long long), st));
    k_fine_totals<FINE_W_BITS><<<dim3(FINE_W / 256, TOT_SLICES), 256, 0, st>>>(
        s->hist.as<unsigned int>(), s->hll.as<uint8_t>(), ngroups, ftot, reinterpret_cast<unsigned int *>(ftot + FINE_W),
        &dsc->nrec);
    k_hll_final<<<1, 1024, 0, st>>>(reinterpret_cast<unsigned int *>(ftot + FINE_W), HLL_REG_BITS, &dsc->est);
    mark(s, 2 * EC_STAGE_PRESCAN + 1);
    EC_CHECK(d2h(s, &hsc, dsc, sizeof(Scalars), st));
    EC_CHECK(host_sync(s, st));
    const uint64_t P = hsc.npos;
    const double est = hsc.est * (hsmask + 1.0);
    // Up to 2^FINE_W_BITS buckets of <= 1100 estimated keys in 3328-slot tables (156 KB: one
    // workgroup per CU), sized exactly by the fine histogram.  Past that (~1.8e7 keys: config
    // 5's 200 Mbp genome has 2e8) a third level splits every fine bucket into 2^sbits
    // fixed-capacity sub-buckets of <= 800 estimated keys in 1664-slot tables (78 KB: two
    // workgroups per CU); measured before: such inputs fell to the HBM table (k_count 130 ms of
    // a 335 ms step at 1.25e9 positions).
    if (kn().verbose)
        fprintf(stderr, "count_wpart: mb %d P %llu est %.0f lens2 %u skew %u maxlocal %u wbv_long %u\n", (int)mb,
                (unsigned long long)hsc.npos, hsc.est, hsc.lens[2], hsc.skew, hsc.maxlocal, hsc.wbv_long);
    if (mb && hsc.wbv_long) {  // reads of several lengths: hash buckets instead
        if (mb_declined) *mb_declined = true;
        return reset();
    }
    if (hsc.lens[2] || hsc.skew || hsc.maxlocal > MAX_LOCAL_EVENT || !P) return reset();
    int sbits = 0;
    // keys per third-level table: <= 800 on hash buckets; <= 400 on minimizer buckets, whose
    // tables hold whole minimizers (~25 k-mers each): config 5's 2^18 tables of mean 763 keys
    // reached 1808, past the 1664 slots (a numpy model of its genome reproduces the five
    // overflowing tables); 2^19 of mean 381 top out at 1421
    // (1024-slot tables of <= 200 keys for the run tables, two workgroups a CU, measured 3x
    // slower on config 5's shape: 355 vs 117 ms)
    const double per3 = mb ? 400.0 : 800.0;
    if (est / FINE_W > 1800.0) {
        while (sbits < 6 && est / (double)(FINE_W << sbits) > per3) sbits++;
        if (est / (double)(FINE_W << sbits) > per3) return reset();
    }
    if (kn().wide_l3 > 0) sbits = std::min(6, kn().wide_l3);
    s->stats.n_reads = nreads;
    s->stats.n_positions = P;
    s->stats.n_distinct_est = (uint64_t)llround(est);

    int bbits = 0;
    int maxb = FINE_W_BITS;  // (EULERHIP_WIDE_MAX_BBITS: tests force bucket overflow)
    if (kn().wide_max_bbits >= 0) maxb = std::max(0, std::min(FINE_W_BITS, kn().wide_max_bbits));
    if (sbits) bbits = FINE_W_BITS;
    while (bbits < maxb && est / (double)(1ull << bbits) > 1100.0) bbits++;
    int fan = 0;
    while ((1 << (fan + 1)) <= REFINE_FANOUT) fan++;
    const int cbits = std::min(bbits, std::min(DS_MAX_CBITS, std::max(1, bbits - fan)));
    const uint64_t Bk = 1ull << bbits, Ck = 1ull << cbits;
    const uint64_t Bt = Bk << sbits;  // tables
    const unsigned int SLOTS = sbits ? 1664u : (unsigned int)SLOTS_W;
    mark(s, 2 * EC_STAGE_COUNT);
    EC_CHECK(s->cnt.ensure(Ck * ngroups * 8));
    EC_CHECK(s->offs.ensure(Ck * ngroups * 8));
    EC_CHECK(s->tot.ensure((Bk + 1) * 8));
    EC_CHECK(s->bstart.ensure((Bk + 1) * 8));
    // record buffers: window records, P of them; runs: the histogram's total (hsc.nrec, exact),
    // and where the bucket pass rolls the runs out of 2-bit codes (third level) the codes go
    // into the refined runs' buffer -- ceil((windows + k - 1) / 16) dwords a run (k_run_ccount).
    // (Both buffers took P 24-B records before: 2 x 30 GB at config 5's rank shape for ~1.3 GB
    // of runs and ~2 GB of codes.)  The two-level case expands the runs into P window records.
    const size_t rbytes = runs ? sizeof(RunWM) : sizeof(RecW);
    const bool second = bbits > cbits;
    const bool direct = runs && sbits && kn().wide_runs != 2;
    const uint64_t NR = runs ? hsc.nrec : P;
    uint64_t b_recs = std::max<uint64_t>(P, 1) * sizeof(RecW), b_recs2 = b_recs;
    if (direct) {
        const uint64_t cbytes = 4 * ((P + NR * (uint64_t)(k - 1)) / 16 + 2 * NR + 64);
        b_recs = b_recs2 = std::max<uint64_t>(std::max<uint64_t>(NR, 1) * sizeof(RunWM), cbytes);
    } else if (runs) {  // the runs' input buffer rin (recs2 after a refine, else recs) takes the windows
        b_recs = std::max<uint64_t>(P, 1) * sizeof(RecW);
        b_recs2 = std::max<uint64_t>(NR, 1) * sizeof(RunWM);
        if (second) std::swap(b_recs, b_recs2);
    }
    EC_CHECK(s->recs.ensure(b_recs));
    if (second || runs) EC_CHECK(s->recs2.ensure(b_recs2));
    s->stats.record_bytes = (uint32_t)rbytes;
    s->stats.n_records = NR;
    k_coarse<FINE_W_BITS><<<grid_for(Ck * ngroups, B, 8192), B, 0, st>>>(s->hist.as<unsigned int>(), ngroups, cbits,
                                                                        s->cnt.as<unsigned long long>());
    EC_CHECK(scan_u64(s, s->cnt.as<unsigned long long>(), s->offs.as<unsigned long long>(), Ck * ngroups));
    k_bucket_totals<FINE_W_BITS><<<grid_for(Bk + 1, B), B, 0, st>>>(ftot, bbits, s->tot.as<unsigned long long>());
    EC_CHECK(scan_u64(s, s->tot.as<unsigned long long>(), s->bstart.as<unsigned long long>(), Bk + 1));
    kmark(s, 1, 0);
    if (runs)
        k_downsweep_wr<<<(unsigned)ngroups, TILE_READS, 0, st>>>(d_off, nreads, k, gsize, ngroups, cbits,
                                                                s->offs.as<unsigned long long>(), s->recs.as<RunWM>(),
                                                                wbv, mbM);
    else if (mb)
        k_downsweep_w<true><<<(unsigned)ngroups, TILE_READS, 0, st>>>(d_reads, d_off, nreads, k, gsize, ngroups, cbits,
                                                                     s->offs.as<unsigned long long>(),
                                                                     s->recs.as<RecW>(), read_base, wbv, mbM);
    else
        k_downsweep_w<false><<<(unsigned)ngroups, TILE_READS, 0, st>>>(d_reads, d_off, nreads, k, gsize, ngroups,
                                                                      cbits, s->offs.as<unsigned long long>(),
                                                                      s->recs.as<RecW>(), read_base, nullptr, 0u);
    kmark(s, 1, 1);
    if (second) {
        const unsigned RS = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(8, 1024 / Ck));
        EC_CHECK(s->gcur.ensure(Bk * 8));
        EC_HIP(hipMemcpyAsync(s->gcur.p, s->bstart.p, Bk * 8, hipMemcpyDeviceToDevice, st));
        kmark(s, 4, 0);
        if (runs)
            k_refine<RunWM, StoreRM, StoreRM><<<dim3((unsigned)Ck, RS), BUCKET_THREADS, 0, st>>>(
                StoreRM{s->recs.as<RunWM>()}, StoreRM{s->recs2.as<RunWM>()}, s->bstart.as<unsigned long long>(),
                s->gcur.as<unsigned long long>(), cbits, bbits);
        else if (mb)
            k_refine<RecWM, StoreWM, StoreWM><<<dim3((unsigned)Ck, RS), BUCKET_THREADS, 0, st>>>(
                StoreWM{s->recs.as<RecWM>()}, StoreWM{s->recs2.as<RecWM>()}, s->bstart.as<unsigned long long>(),
                s->gcur.as<unsigned long long>(), cbits, bbits);
        else
            k_refine<RecW, StoreW, StoreW><<<dim3((unsigned)Ck, RS), BUCKET_THREADS, 0, st>>>(
                StoreW{s->recs.as<RecW>()}, StoreW{s->recs2.as<RecW>()}, s->bstart.as<unsigned long long>(),
                s->gcur.as<unsigned long long>(), cbits, bbits);
        if (sbits && !runs) {  // fine buckets (recs2) -> their sub-buckets (recs), exact (k_split3)
            EC_CHECK(s->bb2.ensure((Bt + 1) * 8));
            const unsigned long long cap3 = kn().wide_l3_cap > 0 ? (unsigned long long)kn().wide_l3_cap : 0ull;
            if (mb)
                k_split3<RecWM><<<(unsigned)Bk, 512, 0, st>>>(s->recs2.as<RecWM>(), s->bstart.as<unsigned long long>(),
                                                              bbits, sbits, s->recs.as<RecWM>(),
                                                              s->bb2.as<unsigned long long>(), cap3, &dsc->overflow);
            else
                k_split3<RecW><<<(unsigned)Bk, 512, 0, st>>>(s->recs2.as<RecW>(), s->bstart.as<unsigned long long>(),
                                                             bbits, sbits, s->recs.as<RecW>(),
                                                             s->bb2.as<unsigned long long>(), cap3, &dsc->overflow);
        }
        kmark(s, 4, 1);
    }
    RecWM *rwin = nullptr;  // runs: the window records of the expansion, bucket bounds in bb2
    RunWM *rdirect = nullptr;  // runs on third-level tables: sorted runs, bounds in run units (bb2)
    uint32_t *wcodes = nullptr;  // ... and their bases as 2-bit codes, table t's from wcodes_tab[t]
    if (runs && sbits && kn().wide_runs != 2) {
        // each fine bucket's runs split into its sub-buckets (run units); the bucket pass rolls
        // the windows out itself (k_bucket_wr)
        RunWM *rin = second ? s->recs2.as<RunWM>() : s->recs.as<RunWM>();
        rdirect = second ? s->recs.as<RunWM>() : s->recs2.as<RunWM>();
        EC_CHECK(s->bb2.ensure((Bt + 1) * 8));
        const unsigned long long cap3 = kn().wide_l3_cap > 0 ? (unsigned long long)kn().wide_l3_cap : 0ull;
        kmark(s, 4, 0);
        k_split3<RunWM><<<(unsigned)Bk, 512, 0, st>>>(rin, s->bstart.as<unsigned long long>(), bbits, sbits, rdirect,
                                                      s->bb2.as<unsigned long long>(), cap3, &dsc->overflow);
        // the sorted runs' bases as 2-bit codes (the refined runs' buffer is free: P 24-B records
        // hold them -- at most 20 code dwords a run)
        EC_CHECK(s->tot.ensure((Bk + 1) * 8));
        EC_CHECK(s->gcur.ensure((Bk + 1) * 8));
        EC_CHECK(s->wcodes_tab.ensure((Bt + 1) * 8));
        k_run_ccount<<<(unsigned)(Bk + 1), 256, 0, st>>>(rdirect, s->bstart.as<unsigned long long>(), k,
                                                        s->tot.as<unsigned long long>(), Bk);
        EC_CHECK(scan_u64(s, s->tot.as<unsigned long long>(), s->gcur.as<unsigned long long>(), Bk + 1));
        wcodes = reinterpret_cast<uint32_t *>(rin);
        k_run_codes<<<(unsigned)Bk, 512, 0, st>>>(rdirect, s->bstart.as<unsigned long long>(),
                                                  s->gcur.as<unsigned long long>(), s->bb2.as<unsigned long long>(),
                                                  sbits, wcodes, s->wcodes_tab.as<unsigned long long>(),
                                                  RunReads{d_reads, d_off, k, mbM, read_base, rpack, rpack_d});
        kmark(s, 4, 1);
    } else if (runs) {
        // each fine bucket's runs sorted by sub-bucket (k_split3_runs, run units), then expanded
        // into its windows' records (k_expand_runs, window units; bb2 = sub-bucket bounds)
        RunWM *rin = second ? s->recs2.as<RunWM>() : s->recs.as<RunWM>();
        RunWM *rsorted = second ? s->recs.as<RunWM>() : s->recs2.as<RunWM>();
        rwin = reinterpret_cast<RecWM *>(rin);  // (the refined runs are dead after the sort)
        EC_CHECK(s->bb2.ensure((Bt + 1) * 8));
        EC_CHECK(s->tot.ensure((Bk + 1) * 8));
        EC_CHECK(s->gcur.ensure((Bk + 1) * 8));
        kmark(s, 4, 0);
        k_run_wsum<<<(unsigned)(Bk + 1), 256, 0, st>>>(rin, s->bstart.as<unsigned long long>(),
                                                      s->tot.as<unsigned long long>(), Bk);
        EC_CHECK(scan_u64(s, s->tot.as<unsigned long long>(), s->gcur.as<unsigned long long>(), Bk + 1));
        k_split3_runs<<<(unsigned)Bk, 512, 0, st>>>(rin, s->bstart.as<unsigned long long>(), bbits, sbits,
                                                    s->gcur.as<unsigned long long>(), rsorted,
                                                    s->bb2.as<unsigned long long>(),
                                                    sbits && kn().wide_l3_cap > 0 ? (unsigned long long)kn().wide_l3_cap
                                                                                  : 0ull,
                                                    &dsc->overflow);
        k_expand_runs<<<(unsigned)Bk, 512, 0, st>>>(rsorted, s->bstart.as<unsigned long long>(),
                                                    s->gcur.as<unsigned long long>(), rwin,
                                                    RunReads{d_reads, d_off, k, mbM, read_base});
        kmark(s, 4, 1);
    }
    mark(s, 2 * EC_STAGE_COUNT + 1);
    mark(s, 2 * EC_STAGE_COMPACT);
    const uint64_t umax = Bt * SLOTS;
    EC_CHECK(s->dkey.ensure(umax * sizeof(K128)));
    EC_CHECK(s->dcnt.ensure(umax * 4));
    EC_CHECK(s->dfc.ensure(umax * 8));
    EC_CHECK(s->dft.ensure(umax * 8));
    if (!s->no_index) EC_CHECK(s->sub.ensure(umax * sizeof(SubSlotW)));
    // minimizer buckets: each bucket's first dense id marked for the tile ranking (k_tile_plan)
    unsigned int *bm = nullptr;
    if (mb && kn().tile_plan != 0) {
        const size_t words = umax / 32 + 2;
        EC_CHECK(s->bmark.ensure(words * 4));
        EC_HIP(hipMemsetAsync(s->bmark.p, 0, words * 4, st));
        bm = s->bmark.as<unsigned int>();
    }
    kmark(s, 2, 0);
#define EC_BUCKET_W(SL, R, SRC, BEG, END)                                                                       \
    k_bucket_w<SL, R><<<(unsigned)Bt, BUCKET_THREADS, 0, st>>>(                                                  \
        SRC, BEG, END, limit, s->dkey.as<K128>(), s->dcnt.as<unsigned int>(), s->dfc.as<unsigned long long>(),    \
        s->dft.as<unsigned long long>(), s->no_index ? nullptr : s->sub.as<SubSlotW>(), &dsc->nsolid,            \
        &dsc->ndistinct, &dsc->overflow, bm)
#define EC_BUCKET_WR(SL, ...)                                                                                    \
    k_bucket_wr<SL, ##__VA_ARGS__><<<(unsigned)Bt, wr_nt, 0, st>>>(                                                 \
        rdirect, s->bb2.as<unsigned long long>(), s->bb2.as<unsigned long long>() + 1, limit, s->dkey.as<K128>(),      \
        s->dcnt.as<unsigned int>(), s->dfc.as<unsigned long long>(), s->dft.as<unsigned long long>(),                \
        s->no_index ? nullptr : s->sub.as<SubSlotW>(), &dsc->nsolid, &dsc->ndistinct, &dsc->overflow, bm,            \
        RunReads{d_reads, d_off, k, mbM, read_base}, wcodes, s->wcodes_tab.as<unsigned long long>())
    // (round 6: two 79-KB workgroups a CU unless EULERHIP_WR_ONE=1 keeps round 5's one 104-KB one)
    const bool wr_one = kn().wr_one != 0;
    const unsigned int wr_nt = wr_one ? WR_NT : 512u;
    if (rdirect && wr_one)
        EC_BUCKET_WR(1664);
    else if (rdirect)
        EC_BUCKET_WR(1664, 512, 1024, LSlotW40);
    else if (sbits && runs)
        EC_BUCKET_W(1664, RecWM, rwin, s->bb2.as<unsigned long long>(), s->bb2.as<unsigned long long>() + 1);
    else if (runs)
        EC_BUCKET_W(SLOTS_W, RecWM, rwin, s->bb2.as<unsigned long long>(), nullptr);
    else if (sbits && mb)
        EC_BUCKET_W(1664, RecWM, s->recs.as<RecWM>(), s->bb2.as<unsigned long long>(),
                    s->bb2.as<unsigned long long>() + 1);
    else if (sbits)
        EC_BUCKET_W(1664, RecW, s->recs.as<RecW>(), s->bb2.as<unsigned long long>(),
                    s->bb2.as<unsigned long long>() + 1);
    else if (mb)
        EC_BUCKET_W(SLOTS_W, RecWM, second ? s->recs2.as<RecWM>() : s->recs.as<RecWM>(),
                    s->bstart.as<unsigned long long>(), nullptr);
    else
        EC_BUCKET_W(SLOTS_W, RecW, second ? s->recs2.as<RecW>() : s->recs.as<RecW>(), s->bstart.as<unsigned long long>(),
                    nullptr);
#undef EC_BUCKET_W
#undef EC_BUCKET_WR
    kmark(s, 2, 1);
    mark(s, 2 * EC_STAGE_COMPACT + 1);
    unsigned long long nruns = 0;
    if (runs) EC_CHECK(d2h(s, &nruns, s->bstart.as<unsigned long long>() + Bk, 8, st));
    EC_CHECK(d2h(s, &hsc, dsc, sizeof(Scalars), st));
    EC_CHECK(host_sync(s, st));
    if (runs) s->stats.n_records = nruns;
    if (hsc.overflow) {  // a bucket outgrew its LDS table: the caller counts on the HBM table
        if (kn().verbose)
            fprintf(stderr, "count_wpart: %u tables overflowed (%llu tables of %u slots, sbits %d, mb %d)\n",
                    hsc.overflow, (unsigned long long)Bt, SLOTS, sbits, (int)mb);
        s->stats.table_retries++;
        return reset();
    }
    U = hsc.nsolid;
    s->stats.n_distinct = hsc.ndistinct;
    s->stats.n_solid = U;
    s->stats.count_path = EC_PATH_PARTITIONED;
    s->stats.n_buckets = (uint32_t)Bt;
    s->stats.table_capacity = umax;
    sidx.table = nullptr;
    sidx.capmask = 0;
    sidx.sub = s->sub.as<SubSlotW>();
    sidx.bbits = bbits + sbits;
    sidx.slots = SLOTS;
    sidx.mb = mb ? 1 : 0;
    sidx.k = k;
    if (2ull * U >= (unsigned long long)CYC) {
        set_error("too many solid k-mers (%u) for 31-bit node ids", U);
        return EC_ERR_CAPACITY;
    }
    s->bmark_ok = bm != nullptr;
    ok = true;
    return EC_OK;
}

int phase_count_w(ec_session *s, const uint8_t *d_reads, const uint64_t *d_off, uint64_t nreads, uint64_t read_base,
                  int k, long long limit, unsigned int &U, SolidIndexW &sidx) {
    if (nreads + read_base > (1ull << 32)) {
        set_error("global read ids reach %llu >= 2^32", (unsigned long long)(nreads + read_base));
        return EC_ERR_ARG;
    }
    bool ok = false;
    {
        // minimizer buckets for k <= 52 (count_wide.h; EULERHIP_WIDE_MB=0: hash buckets)
        bool declined = false;
        // (config-5 rank shape: 141 ms a step against 169 ms on mix128 buckets --
        // profiles/r04_l_config5_rank_shape_minimizer_buckets.json)
        const bool mb = k <= WMB_MAX_K && kn().wide_mb != 0;
        EC_CHECK(phase_count_wpart(s, d_reads, d_off, nreads, read_base, k, limit, U, sidx, ok, mb, &declined));
        if (declined) EC_CHECK(phase_count_wpart(s, d_reads, d_off, nreads, read_base, k, limit, U, sidx, ok));
    }
    if (ok) return EC_OK;
    s->stats.n_reads = nreads;
    hipStream_t st = s->stream;
    const unsigned B = 256;
    Scalars *dsc = s->scal.as<Scalars>();
    Scalars hsc;
    mark(s, 2 * EC_STAGE_PRESCAN);
    EC_CHECK(s->hll.ensure(HLL_M * 4));
    EC_HIP(hipMemsetAsync(s->hll.p, 0, HLL_M * 4, st));
    if (nreads) {
        k_prescan_w<<<grid_for(nreads, B, 4096), B, 0, st>>>(d_reads, d_off, nreads, k, s->hll.as<unsigned int>(),
                                                            &dsc->npos, &dsc->bad);
        k_hll_final<<<1, 1024, 0, st>>>(s->hll.as<unsigned int>(), HLL_BITS, &dsc->est);
    }
    mark(s, 2 * EC_STAGE_PRESCAN + 1);
    EC_CHECK(d2h(s, &hsc, dsc, sizeof(Scalars), st));
    EC_CHECK(host_sync(s, st));
    if (hsc.bad != ~0ull) {
        uint8_t byte = 0;
        hipMemcpy(&byte, d_reads + hsc.bad, 1, hipMemcpyDeviceToHost);
        set_error("byte %llu (0x%02x) outside {A,C,G,T,N}", (unsigned long long)hsc.bad, byte);
        return EC_ERR_ALPHABET;
    }
    const uint64_t P = nreads ? hsc.npos : 0;
    s->stats.n_positions = P;
    const double est = nreads ? hsc.est : 0.0;
    s->stats.n_distinct_est = (uint64_t)llround(est);
    uint64_t cap = 1024;
    const double want = std::min((double)P, 1.05 * est) * 1.6 + 1024;
    while ((double)cap < want) cap <<= 1;
    for (int attempt = 0;; attempt++) {
        EC_CHECK(s->table.ensure(cap * sizeof(SlotW)));
        mark(s, 2 * EC_STAGE_COUNT);
        k_table_clear_w<<<grid_for(cap, B, 8192), B, 0, st>>>(s->table.as<SlotW>(), cap);
        EC_HIP(hipMemsetAsync(&dsc->overflow, 0, 4, st));
        if (nreads) {
            kmark(s, 3, 0);
            k_count_w<<<grid_for(nreads, B), B, 0, st>>>(d_reads, d_off, nreads, k, s->table.as<SlotW>(), cap - 1,
                                                        &dsc->overflow, read_base);
            kmark(s, 3, 1);
        }
        mark(s, 2 * EC_STAGE_COUNT + 1);
        EC_CHECK(d2h(s, &hsc.overflow, &dsc->overflow, 4, st));
        EC_CHECK(host_sync(s, st));
        if (!hsc.overflow) break;
        if (attempt >= 4) {
            set_error("hash table overflow at capacity %llu", (unsigned long long)cap);
            return EC_ERR_CAPACITY;
        }
        cap <<= 2;
        s->stats.table_retries++;
    }
    return finish_wide(s, cap, limit, U, sidx);
}

// The owner merge's dense set (U ids in table order) reordered by minimizer (shard.h k_wplace /
// k_wpermute), the minimizers' first ids marked for the partitioned finish's tiles: the
// gathered ids of 128-bit keys get the locality minimizer owners give (round 5)
int order_by_minimizer_w(ec_session *s, unsigned int U) {
    hipStream_t st = s->stream;
    const unsigned B = 256;
    if (!U) return EC_OK;
    EC_CHECK(s->skeys.ensure((size_t)U * 8));
    EC_CHECK(s->skeys2.ensure((size_t)U * 8));
    EC_CHECK(s->svals.ensure((size_t)U * 4));
    EC_CHECK(s->svals2.ensure((size_t)U * 4));
    k_wplace<<<grid_for(U, B), B, 0, st>>>(s->dkey.as<K128>(), U, s->k, s->skeys.as<unsigned long long>(),
                                           s->svals.as<unsigned int>());
    EC_CHECK(sort_pairs(s, s->skeys.as<unsigned long long>(), s->skeys2.as<unsigned long long>(),
                        s->svals.as<unsigned int>(), s->svals2.as<unsigned int>(), U));
    // permuted into the count-phase record buffers (free on the owner side), then swapped in
    EC_CHECK(s->recs.ensure((size_t)U * sizeof(K128)));
    EC_CHECK(s->recs2.ensure((size_t)U * 16));
    EC_CHECK(s->mbid2.ensure((size_t)U * 4));
    unsigned long long *nfc = s->recs2.as<unsigned long long>(), *nft = nfc + U;
    k_wpermute<<<grid_for(U, B), B, 0, st>>>(s->svals2.as<unsigned int>(), U, s->dkey.as<K128>(),
                                             s->dcnt.as<unsigned int>(), s->dfc.as<unsigned long long>(),
                                             s->dft.as<unsigned long long>(), s->recs.as<K128>(),
                                             s->mbid2.as<unsigned int>(), nfc, nft);
    std::swap(s->dkey, s->recs);
    std::swap(s->dcnt, s->mbid2);
    EC_CHECK(s->dfc.ensure((size_t)U * 8));
    EC_CHECK(s->dft.ensure((size_t)U * 8));
    EC_HIP(hipMemcpyAsync(s->dfc.p, nfc, (size_t)U * 8, hipMemcpyDeviceToDevice, st));
    EC_HIP(hipMemcpyAsync(s->dft.p, nft, (size_t)U * 8, hipMemcpyDeviceToDevice, st));
    if (kn().tile_plan != 0) {
        const unsigned int words = U / 32 + 2;
        EC_CHECK(s->bmark.ensure((size_t)words * 4));
        k_wmarks<<<grid_for(words, B), B, 0, st>>>(s->skeys2.as<unsigned long long>(), U, s->bmark.as<unsigned int>(),
                                                   words);
        s->seg_marks = U;
    }
    return EC_OK;
}

int phase_merge_w(ec_session *s, const AggW *d_agg, uint64_t n, long long limit, unsigned int &U, SolidIndexW &sidx) {
    hipStream_t st = s->stream;
    const unsigned B = 256;
    Scalars *dsc = s->scal.as<Scalars>();
    Scalars hsc;
    // the table for the distinct keys (HyperLogLog of the records' keys, +-2.3 %), not for the
    // records: a rank's merge sees each key once per source (a table past 0.45 load retries x4)
    double keys = (double)n;
    if (n >= (1u << 20)) {
        constexpr int HB = HLL_REG_BITS;
        EC_CHECK(s->ftot.ensure((1 << HB) * 4));
        unsigned int *hreg = s->ftot.as<unsigned int>();
        EC_HIP(hipMemsetAsync(hreg, 0, (1 << HB) * 4, st));
        k_hll_aggw<<<256, B, 0, st>>>(d_agg, n, HB, hreg);
        k_hll_final<<<1, 1024, 0, st>>>(hreg, HB, &dsc->est);
        double est = 0;
        EC_CHECK(d2h(s, &est, &dsc->est, sizeof(double), st));
        EC_CHECK(host_sync(s, st));
        keys = std::min((double)n, est * 1.1 + 1024.0);
    }
    uint64_t cap = 1024;
    while (cap < (uint64_t)(2.2 * keys) + 1024) cap <<= 1;
    for (int attempt = 0;; attempt++) {
        EC_CHECK(s->table.ensure(cap * sizeof(SlotW)));
        mark(s, 2 * EC_STAGE_COUNT);
        k_table_clear_w<<<grid_for(cap, B, 8192), B, 0, st>>>(s->table.as<SlotW>(), cap);
        EC_HIP(hipMemsetAsync(&dsc->overflow, 0, 4, st));
        if (n) k_merge_agg_w<<<grid_for(n, B), B, 0, st>>>(d_agg, n, s->table.as<SlotW>(), cap - 1, &dsc->overflow);
        mark(s, 2 * EC_STAGE_COUNT + 1);
        EC_CHECK(d2h(s, &hsc.overflow, &dsc->overflow, 4, st));
        EC_CHECK(host_sync(s, st));
        if (!hsc.overflow) break;
        if (attempt >= 4) {
            set_error("merge table overflow at capacity %llu", (unsigned long long)cap);
            return EC_ERR_CAPACITY;
        }
        cap <<= 2;
        s->stats.table_retries++;
    }
    EC_CHECK(finish_wide(s, cap, limit, U, sidx, std::max<uint64_t>(n, 1)));
    // an owner merge (no lookup index wanted) on minimizer owners: ids in minimizer order
    if (s->no_index && s->owner_rule == 0 && merge_wmb(s->k) && !(s->flags & EC_FLAG_GENERAL)) {
        EC_CHECK(order_by_minimizer_w(s, U));
        sidx.table = nullptr;  // (the table's ids are the pre-order ones)
    }
    return EC_OK;
}

// palindrome flags of the canonical keys (k_upal).  Odd k over A/C/G/T has no palindromic
// k-mer (the middle base would be its own complement): the flags are a fill, not a pass over the
// keys (config 5: 0.64 ms of reading 3.2 GB of keys for nothing)
template <typename Ops>
inline int launch_upal(hipStream_t st, const typename Ops::K *dkey, unsigned int U, int k, uint8_t *upal,
                       unsigned int *npal) {
    if (!U) return EC_OK;
    if ((k & 1) && (std::is_same<Ops, Ops64>::value || std::is_same<Ops, OpsW>::value)) {
        EC_HIP(hipMemsetAsync(upal, 0, U, st));
        return EC_OK;
    }
    k_upal<Ops><<<grid_for(U, 256), 256, 0, st>>>(dkey, U, k, upal, npal);
    return EC_OK;
}

// Links by the (k-1)-mer half-edge join (join_w.h), 128-bit (OpsW) or 64-bit (Ops64) keys.
// gate: a device flag set when a level region or a join table overflowed; the caller then
// launches k_neighbors / k_succ gated on it (they return at once unless it is set).
template <typename Ops> struct JoinT;
template <> struct JoinT<OpsW> {
    using R = RecJ;
    using S = StoreJ;
    static void emit_l1(const K128 *d, unsigned U, int k, const uint8_t *up, int lb, uint64_t fc, unsigned long long *gc,
                        R *o, unsigned *ov, hipStream_t st) {
        k_half_emit_l1<K128, R><<<grid_for(U, 1024, 2048), 1024, 0, st>>>(d, U, k, up, lb, fc, gc, o, ov);
    }
    template <bool ODD>
    static void join(unsigned nb, const R *r, const unsigned long long *bb, const unsigned long long *be,
                     const uint8_t *up, unsigned *succ, unsigned *ov, hipStream_t st) {
        k_half_join<2048, 512, ODD><<<nb, 512, 0, st>>>(r, bb, be, up, succ, ov);
    }
};
struct JoinTM {  // 128-bit keys on minimizer-bucketed ids: junctions bucketed by their minimizer
    using R = RecJM;
    using S = StoreJM;
    static void emit_l1(const K128 *d, unsigned U, int k, const uint8_t *up, int lb, uint64_t fc, unsigned long long *gc,
                        R *o, unsigned *ov, hipStream_t st) {
        k_half_emit_l1<K128, R><<<grid_for(U, 1024, 2048), 1024, 0, st>>>(d, U, k, up, lb, fc, gc, o, ov);
    }
    template <bool ODD>
    static void join(unsigned nb, const R *r, const unsigned long long *bb, const unsigned long long *be,
                     const uint8_t *up, unsigned *succ, unsigned *ov, hipStream_t st) {
        k_half_join<2048, 512, ODD, RecJM><<<nb, 512, 0, st>>>(r, bb, be, up, succ, ov);
    }
};
template <> struct JoinT<Ops64> {
    using R = RecJ64;
    using S = StoreJ64;
    static void emit_l1(const unsigned long long *d, unsigned U, int k, const uint8_t *up, int lb, uint64_t fc,
                        unsigned long long *gc, R *o, unsigned *ov, hipStream_t st) {
        k_half_emit_l1<unsigned long long, R><<<grid_for(U, 1024, 2048), 1024, 0, st>>>(d, U, k, up, lb, fc, gc, o, ov);
    }
    template <bool ODD>
    static void join(unsigned nb, const R *r, const unsigned long long *bb, const unsigned long long *be,
                     const uint8_t *up, unsigned *succ, unsigned *ov, hipStream_t st) {
        k_half_join64<2048, 512, ODD><<<nb, 512, 0, st>>>(r, bb, be, up, succ, ov);
    }
};

template <typename Ops, typename J = JoinT<Ops>>
int links_join(ec_session *s, int k, unsigned int U, bool &ok, const unsigned int *&gate) {
    using R = typename J::R;
    using S = typename J::S;
    ok = false;
    hipStream_t st = s->stream;
    const unsigned B = 256;
    Scalars *dsc = s->scal.as<Scalars>();
    const uint64_t N = 2ull * U;
    // final buckets of <= 900 (k-1)-mer groups (~U of them) in 2048-slot tables; levels of <= 256
    int bt = 1;
    while ((double)U / (double)(1ull << bt) > 900.0) bt++;
    std::vector<int> lv;
    for (int rem = bt; rem > 0; rem -= std::min(8, rem)) lv.push_back(std::min(8, rem));
    uint64_t needA = 0, needB = 0, nbmax = 1;
    std::vector<uint64_t> fc(lv.size());
    for (size_t l = 0, cb = 0; l < lv.size(); l++) {
        cb += lv[l];
        const uint64_t nb = 1ull << cb, mean = N / nb;
        fc[l] = kn().join_cap > 0 ? (uint64_t)kn().join_cap : mean + mean * 3 / 10 + 1024;
        (l & 1 ? needA : needB) = std::max(l & 1 ? needA : needB, nb * fc[l]);
        nbmax = std::max(nbmax, nb);
    }
    EC_CHECK(s->recs.ensure(needA * sizeof(R)));
    EC_CHECK(s->recs2.ensure(needB * sizeof(R)));
    EC_CHECK(s->bb2.ensure(2 * nbmax * 8));
    EC_CHECK(s->gcur.ensure(nbmax * 8));
    EC_CHECK(s->tmp.ensure(16));
    unsigned int *flags = s->tmp.as<unsigned int>();  // [1]: a level region or a join table overflowed
    unsigned long long *ibeg = s->bb2.as<unsigned long long>(), *iend = ibeg + nbmax;
    EC_HIP(hipMemsetAsync(flags, 0, 8, st));
    const typename Ops::K *dkey = s->dkey.as<typename Ops::K>();
    EC_CHECK(launch_upal<Ops>(st, dkey, U, k, s->upal.as<uint8_t>(), &dsc->npal));
    R *src = s->recs.as<R>(), *dst = s->recs2.as<R>();
    // level 0 fused with the emit (k_half_emit_l1), its regions in dst
    const uint64_t nb0 = 1ull << lv[0];
    k_cursor_init<<<grid_for(nb0, B, 8192), B, 0, st>>>(s->gcur.as<unsigned long long>(), nb0, fc[0]);
    J::emit_l1(dkey, U, k, s->upal.as<uint8_t>(), lv[0], fc[0], s->gcur.as<unsigned long long>(), dst, &flags[1], st);
    k_level3_ends<<<grid_for(nb0, B, 8192), B, 0, st>>>(s->gcur.as<unsigned long long>(), nb0, fc[0], ibeg, iend);
    std::swap(src, dst);
    int cb = lv[0];
    for (size_t l = 1; l < lv.size(); l++) {
        const uint64_t nc = 1ull << cb, nb = 1ull << (cb + lv[l]);
        k_cursor_init<<<grid_for(nb, B, 8192), B, 0, st>>>(s->gcur.as<unsigned long long>(), nb, fc[l]);
        const unsigned rs = (unsigned)std::max<uint64_t>(1, 1024 / nc);
        k_refine<R, S, S><<<dim3((unsigned)nc, rs), BUCKET_THREADS, 0, st>>>(
            S{src}, S{dst}, nullptr, s->gcur.as<unsigned long long>(), cb, cb + lv[l], fc[l], &flags[1], ibeg, iend);
        k_level3_ends<<<grid_for(nb, B, 8192), B, 0, st>>>(s->gcur.as<unsigned long long>(), nb, fc[l], ibeg, iend);
        std::swap(src, dst);
        cb += lv[l];
    }
    EC_HIP(hipMemsetAsync(s->succ.p, 0xFF, N * 4, st));
    if (k & 1)
        J::template join<true>((unsigned)(1ull << cb), src, ibeg, iend, s->upal.as<uint8_t>(), s->succ.as<unsigned int>(),
                               &flags[1], st);
    else
        J::template join<false>((unsigned)(1ull << cb), src, ibeg, iend, s->upal.as<uint8_t>(),
                                s->succ.as<unsigned int>(), &flags[1], st);
    // no host round trip: the caller's probe kernels run gated on flags[1] (a level region or a
    // join table that overflowed) and then rewrite every successor
    gate = &flags[1];
    ok = true;
    return EC_OK;
}

// Links joined inside the count's minimizer tables (join_local.h): keys on tables of ids grouped
// by table -- the super-k-mer count's minimizer tables (64-bit), the wide minimizer count's
// (128-bit).  ok = false: not such an index (the caller takes links_join).
template <typename Index>
inline int jl_bits(const Index &) { return -1; }
template <>
inline int jl_bits<SolidIndex>(const SolidIndex &x) { return x.sub && x.sk && !x.npb && !x.bijk ? x.bbits : -1; }
template <>
inline int jl_bits<SolidIndexW>(const SolidIndexW &x) { return x.sub && x.mb ? x.bbits : -1; }

template <typename Ops, typename Index>
int links_local(ec_session *s, int k, unsigned int U, const Index &sidx, bool &ok, const unsigned int *&gate) {
    using K = typename Ops::K;
    using R = typename JLRec<K>::R;
    ok = false;
    int bits = jl_bits(sidx);
    if (bits < 1 || bits > 22 || k < SK_M + 2) return EC_OK;
    // (tests: tables finer or coarser than the count's -- ids not grouped by table, the gate opens)
    if (kn().jl_bits_delta) bits = std::max(1, std::min(22, bits + kn().jl_bits_delta));
    const unsigned int ntab = 1u << bits;
    // a table's junction groups ~ its keys (plus the foreign records sent to it): tables of mean
    // <= ~700 keys in 2048 slots, <= ~1500 in 4096 (an overflowing one opens the gate)
    const double mean = (double)U / ntab;
    const int slots = mean <= 700.0 ? 2048 : mean <= 1500.0 ? 4096 : 0;
    if (!slots) return EC_OK;
    hipStream_t st = s->stream;
    const unsigned B = 256;
    Scalars *dsc = s->scal.as<Scalars>();
    const uint64_t N = 2ull * U;
    // foreign records: ~2 / (w + 1) of the 2U (7 % at k = 31, 3 % at k = 51); room for a third
    const unsigned int fcap = kn().jl_fcap > 0 ? ((unsigned int)kn().jl_fcap / JL_NCTR + 1) * JL_NCTR
                                               : (U / 3 / JL_NCTR + 64) * JL_NCTR;
    EC_CHECK(s->jl_kof.ensure((size_t)U * 4));
    EC_CHECK(s->jl_rs.ensure((size_t)ntab * 4));
    EC_CHECK(s->jl_re.ensure((size_t)ntab * 4));
    EC_CHECK(s->jl_cnt.ensure(((size_t)ntab + 1) * 4));
    EC_CHECK(s->jl_off.ensure(((size_t)ntab + 1) * 4));
    EC_CHECK(s->jl_flag.ensure((size_t)(JL_NCTR + 1) * JL_CSTRIDE * 4));
    EC_CHECK(s->recs.ensure((size_t)fcap * sizeof(R)));
    EC_CHECK(s->recs2.ensure((size_t)fcap * sizeof(R)));
    // [1]: the gate; [JL_CSTRIDE (r + 1)]: foreign records of region r
    unsigned int *flags = s->jl_flag.as<unsigned int>(), *fctr = flags + JL_CSTRIDE;
    unsigned int *cnt = s->jl_cnt.as<unsigned int>(), *off = s->jl_off.as<unsigned int>();
    const K *dkey = s->dkey.as<K>();
    uint8_t *upal = s->upal.as<uint8_t>();
    // (odd k: no palindromic k-mer, the flags a fill in the same launch; even k: k_upal)
    k_jl_init<<<grid_for(N, B, 4096), B, 0, st>>>(flags, (JL_NCTR + 1) * JL_CSTRIDE, s->jl_rs.as<unsigned int>(), cnt,
                                                 ntab, s->succ.as<unsigned int>(), N, (k & 1) ? upal : nullptr, U);
    if (!(k & 1)) EC_CHECK(launch_upal<Ops>(st, dkey, U, k, upal, &dsc->npal));
    k_jl_scan<K><<<grid_for(U, B, 8192), B, 0, st>>>(dkey, U, k, bits, upal, s->jl_kof.as<unsigned int>(), s->recs.as<R>(),
                                                     fctr, fcap, cnt, s->jl_rs.as<unsigned int>(),
                                                     s->jl_re.as<unsigned int>(), &flags[1]);
    k_jl_edges<<<grid_for(U / 64 + 2, B, 4096), B, 0, st>>>(s->jl_kof.as<unsigned int>(), U, s->jl_rs.as<unsigned int>(),
                                                           s->jl_re.as<unsigned int>(), &flags[1]);
    EC_CHECK(scan_excl_u32(s, cnt, off, (size_t)ntab + 1));
    k_jl_scatter<R><<<grid_for(fcap, B, 4096), B, 0, st>>>(s->recs.as<R>(), fctr, fcap, off, cnt, s->recs2.as<R>());
    // (4096 slots: 96 KB of 128-bit slots, one workgroup a CU -- 512 threads to hide the probes)
#define EC_JL_JOIN(SL, ODD)                                                                                        \
    k_jl_join<K, SL, SL / 8, ODD><<<ntab, SL / 8, 0, st>>>(dkey, s->jl_kof.as<unsigned int>(), s->jl_rs.as<unsigned int>(), \
                                                     s->jl_re.as<unsigned int>(), k, upal, s->recs2.as<R>(), off,     \
                                                     s->succ.as<unsigned int>(), &flags[1])
    if (slots == 2048) {
        if (k & 1) EC_JL_JOIN(2048, true);
        else EC_JL_JOIN(2048, false);
    } else {
        if (k & 1) EC_JL_JOIN(4096, true);
        else EC_JL_JOIN(4096, false);
    }
#undef EC_JL_JOIN
    EC_HIP(hipGetLastError());
    gate = &flags[1];
    ok = true;
    return EC_OK;
}

// rank_tile.h (2): the super list srec (M chains, SIDX[head] = index) linked and ranked by the
// weighted ruling set; per chain its path key / rank (rt_pks / rt_rks), paths' and cycles'
// length / min first event at their key nodes (PL / PM)
int rank_supers(ec_session *s, unsigned int M, unsigned int N, unsigned int &nr, int &rounds,
                bool pre_init = false, const unsigned int *sidx = nullptr) {
    hipStream_t st = s->stream;
    const unsigned B = 256;
    Scalars *dsc = s->scal.as<Scalars>();
    Scalars hsc{};
    SuperRec *srec = s->rt_srec.as<SuperRec>();
    // (sidx: head node -> super index; the look-back compaction's LH serves, being that at heads)
    const unsigned int *SIDX = sidx ? sidx : s->rt_sidx.as<unsigned int>();
    const size_t cap = std::max<size_t>(M, 1);
    EC_CHECK(s->rt_snrec.ensure(cap * sizeof(SNodeRec)));
    EC_CHECK(s->rt_hasp.ensure(cap));
    EC_CHECK(s->rt_pks.ensure(cap * 4));
    EC_CHECK(s->rt_rks.ensure(cap * 4));
    EC_CHECK(s->rid.ensure(cap * 8));
    EC_CHECK(s->rlist.ensure(cap * 4));
    EC_CHECK(s->nextR.ensure(cap * 4));
    EC_CHECK(s->st0.ensure(cap * sizeof(RJump)));
    EC_CHECK(s->st1.ensure(cap * sizeof(RJump)));
    EC_CHECK(s->rbc.ensure(((cap + RULER_CHUNK - 1) / RULER_CHUNK) * 8 + 8));
    SNodeRec *snrec = s->rt_snrec.as<SNodeRec>();
    if (!pre_init) EC_HIP(hipMemsetAsync(s->rt_hasp.p, 0, M, st));  // (pre_init: k_tile_compact did these)
    k_super_link<<<grid_for(M, B), B, 0, st>>>(srec, M, SIDX, snrec, s->rt_hasp.as<uint8_t>());
    if (!pre_init) {
        EC_HIP(hipMemsetAsync(s->rid.p, 0xFF, (size_t)M * 8, st));
        EC_HIP(hipMemsetAsync(&dsc->nr, 0, 4, st));
        EC_HIP(hipMemsetAsync(&dsc->nvisited, 0, 8, st));
    }
    unsigned int masks[4] = {15u, 3u, 1u, 0u};
    if (kn().sruler_mask > 0) masks[0] = (unsigned int)kn().sruler_mask;  // (A/B: first-pass ruler density)
    unsigned int r0 = 0;
    const unsigned int nblk = (M + RULER_CHUNK - 1) / RULER_CHUNK;
    for (int it = 0; it < 4; it++) {
        k_srulers_count<<<nblk, B, 0, st>>>(s->rt_hasp.as<uint8_t>(), M, masks[it], it == 0, s->rid.as<uint2>(),
                                            s->rbc.as<unsigned int>());
        EC_CHECK(scan_incl_u32(s, s->rbc.as<unsigned int>(), s->rbc.as<unsigned int>() + nblk, nblk));
        k_srulers<<<nblk, B, 0, st>>>(s->rt_hasp.as<uint8_t>(), M, masks[it], it == 0, s->rbc.as<unsigned int>() + nblk,
                                      &dsc->nr, s->rid.as<uint2>(), s->rlist.as<unsigned int>());
        k_rulers_total<<<1, 1, 0, st>>>(s->rbc.as<unsigned int>() + nblk, nblk, &dsc->nr);
        k_walk_s<<<2048, B, 0, st>>>(snrec, s->rlist.as<unsigned int>(), r0, &dsc->nr, masks[it], s->rid.as<uint2>(),
                                     s->nextR.as<unsigned int>(), s->st0.as<RJump>(), &dsc->nvisited, srec);
        EC_CHECK(d2h(s, &hsc, dsc, sizeof(Scalars), st));
        EC_CHECK(host_sync(s, st));
        r0 = hsc.nr;
        if (hsc.nvisited >= M) break;
    }
    nr = hsc.nr;
    if (hsc.nvisited != M) {
        set_error("ruling set covered %llu of %u chains", (unsigned long long)hsc.nvisited, M);
        return EC_ERR_STATE;
    }
    k_rjump_init<<<grid_for(nr, B), B, 0, st>>>(s->nextR.as<unsigned int>(), nr, s->st0.as<RJump>());
    rounds = 1;
    while ((1ull << (rounds - 1)) < (unsigned long long)nr) rounds++;
    rounds = std::min(rounds + 1, 63);
    RJump *bufs[2] = {s->st0.as<RJump>(), s->st1.as<RJump>()};
    // (the rounds only raise their flags: clear what an unconverged queued ranking left)
    EC_HIP(hipMemsetAsync(dsc->active, 0, sizeof(dsc->active), st));
    for (int r = 0; r < rounds; r++)
        k_rjump<<<grid_for(nr, B), B, 0, st>>>(bufs[r & 1], bufs[(r + 1) & 1], nr, N, r ? &dsc->active[r - 1] : nullptr,
                                              &dsc->active[r], &dsc->final_sel, (unsigned)((r + 1) & 1));
    k_finalize_s<<<grid_for(M, B), B, 0, st>>>(snrec, srec, s->rid.as<uint2>(), s->rlist.as<unsigned int>(), bufs[0],
                                              bufs[1], &dsc->final_sel, &dsc->active[rounds - 1], M,
                                              s->rt_pks.as<unsigned int>(), s->rt_rks.as<unsigned int>(),
                                              s->PL.as<unsigned int>(), s->PM.as<unsigned long long>());
    k_cycle_len_s<<<grid_for(nr, B), B, 0, st>>>(s->nextR.as<unsigned int>(), s->rlist.as<unsigned int>(), srec, bufs[0],
                                                bufs[1], &dsc->final_sel, &dsc->active[rounds - 1], nr,
                                                s->PL.as<unsigned int>(), s->PM.as<unsigned long long>());
    return EC_OK;
}

// rank_supers without host read-backs: the chain count M and the ruler count stay on the device
// (dM, Scalars::nr), grids are sized by the node count N >= M and read the counts in-kernel,
// one ruler pass only (mask 15 plus every head), Wyllie rounds for N rulers (rounds past
// convergence exit at once).  The whole ranking is queued while the device still runs the links:
// after a read-back the host issued these ~25 launches slower than the device ran them
// (~0.25 ms from the walk to finalize on the headline).  Chains no ruler reached (a cycle of
// chains without a sampled one) are caught by the caller's next scalar read (nvisited < M),
// which redoes the ranking with rank_supers.  Needs k_tile_compact's initialisation (pre_init).
int rank_supers_async(ec_session *s, unsigned int N, const unsigned long long *dM, int &rounds,
                      unsigned int mcap = 0, const unsigned int *sidx = nullptr) {
    // mcap: a bound of the chain count known on the host (the partitioned finish's gathered
    // list) -- grids and Wyllie rounds sized by it instead of the node count N, which stays the
    // cycle bound of the jumps (j.s < N)
    const unsigned int G = mcap ? mcap : N;
    hipStream_t st = s->stream;
    const unsigned B = 256;
    Scalars *dsc = s->scal.as<Scalars>();
    SuperRec *srec = s->rt_srec.as<SuperRec>();
    // (buffers sized by N, not by the chain count, when the count is only on the device: a count a
    // little above the last call's would reallocate them; with mcap, by it with part_rank's spare
    // -- the gathered list of the partitioned finish is far below its node count)
    const size_t cap = mcap ? (size_t)mcap + 4096 : std::max<size_t>(N, 1);
    const unsigned int spare = mcap ? 16u : 0u;
    EC_CHECK(s->rt_snrec.ensure(cap * sizeof(SNodeRec), spare));
    EC_CHECK(s->rt_pks.ensure(cap * 4, spare));
    EC_CHECK(s->rt_rks.ensure(cap * 4, spare));
    EC_CHECK(s->rlist.ensure(cap * 4, spare));
    EC_CHECK(s->nextR.ensure(cap * 4, spare));
    EC_CHECK(s->rbc.ensure(((cap + RULER_CHUNK - 1) / RULER_CHUNK) * 8 + 8, spare));
    SNodeRec *snrec = s->rt_snrec.as<SNodeRec>();
    const unsigned int *dnr = &dsc->nr;
    const unsigned int gs = std::min(grid_for(G, B), 4096u);  // grid-stride grids over <= G items
    k_super_link<<<gs, B, 0, st>>>(srec, 0, sidx ? sidx : s->rt_sidx.as<unsigned int>(), snrec,
                                   s->rt_hasp.as<uint8_t>(), dM);
    const unsigned int smask = kn().sruler_mask > 0 ? (unsigned int)kn().sruler_mask : 15u;
    const unsigned int nblk = (G + RULER_CHUNK - 1) / RULER_CHUNK;
    k_srulers_count<<<nblk, B, 0, st>>>(s->rt_hasp.as<uint8_t>(), 0, smask, 1, s->rid.as<uint2>(),
                                        s->rbc.as<unsigned int>(), dM);
    EC_CHECK(scan_incl_u32(s, s->rbc.as<unsigned int>(), s->rbc.as<unsigned int>() + nblk, nblk));
    k_srulers<<<nblk, B, 0, st>>>(s->rt_hasp.as<uint8_t>(), 0, smask, 1, s->rbc.as<unsigned int>() + nblk, &dsc->nr,
                                  s->rid.as<uint2>(), s->rlist.as<unsigned int>(), dM);
    k_rulers_total<<<1, 1, 0, st>>>(s->rbc.as<unsigned int>() + nblk, nblk, &dsc->nr);
    k_walk_s<<<2048, B, 0, st>>>(snrec, s->rlist.as<unsigned int>(), 0, &dsc->nr, smask, s->rid.as<uint2>(),
                                 s->nextR.as<unsigned int>(), s->st0.as<RJump>(), &dsc->nvisited, srec);
    // rulers <= chains <= N: rounds for N (a round after convergence returns at its first load)
    const unsigned int gr = std::min(grid_for(G / (kn().rj_div > 0 ? (unsigned)kn().rj_div : 8u) + 1, B), 2048u);
    k_rjump_init<<<gr, B, 0, st>>>(s->nextR.as<unsigned int>(), 0, s->st0.as<RJump>(), dnr);
    rounds = 1;
    while ((1ull << (rounds - 1)) < (unsigned long long)G) rounds++;
    rounds = std::min(rounds + 1, 63);
    if (s->spec_rounds > 0 && s->spec_rounds < rounds) rounds = s->spec_rounds;
    RJump *bufs[2] = {s->st0.as<RJump>(), s->st1.as<RJump>()};
    for (int r = 0; r < rounds; r++)
        k_rjump<<<gr, B, 0, st>>>(bufs[r & 1], bufs[(r + 1) & 1], 0, N, r ? &dsc->active[r - 1] : nullptr,
                                  &dsc->active[r], &dsc->final_sel, (unsigned)((r + 1) & 1), dnr);
    k_finalize_s<<<gs, B, 0, st>>>(snrec, srec, s->rid.as<uint2>(), s->rlist.as<unsigned int>(), bufs[0], bufs[1],
                                   &dsc->final_sel, &dsc->active[rounds - 1], 0, s->rt_pks.as<unsigned int>(),
                                   s->rt_rks.as<unsigned int>(), s->PL.as<unsigned int>(),
                                   s->PM.as<unsigned long long>(), dM);
    k_cycle_len_s<<<gr, B, 0, st>>>(s->nextR.as<unsigned int>(), s->rlist.as<unsigned int>(), srec, bufs[0], bufs[1],
                                    &dsc->final_sel, &dsc->active[rounds - 1], 0, s->PL.as<unsigned int>(),
                                    s->PM.as<unsigned long long>(), dnr);
    return EC_OK;
}

// contig characters -> 2-bit codes (A C G T = 0..3, pack4's mapping), 16 characters a thread,
// up to *total (the contigs' offsets' last entry) of them; the bytes past it are padding
__global__ void __launch_bounds__(256) k_pack_chars(const uint4 *chars, const unsigned long long *total, uint64_t cap16,
                                                    uint32_t *codes) {
    const uint64_t n16 = min<uint64_t>((*total + 15) / 16, cap16);
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < n16; t += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 v = chars[t];
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
        uint32_t out = 0;
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t x = ((w[u] >> 1) ^ (w[u] >> 2)) & 0x03030303u;  // A C G T -> 0 1 2 3 per byte
            const uint32_t y = x | (x >> 6);
            out |= ((y | (y >> 12)) & 0xFFu) << (8 * u);
        }
        codes[t] = out;
    }
}

// the rounds a ranking used (the last round that still moved a pointer + 1), for the next
// call's speculation; 0 when the last round still moved one (not converged)
constexpr unsigned int OCOPY_MIN = 1u << 16;  // contigs past which results copy on the output stream
int rounds_used(const Scalars &h, int rounds) {
    if (rounds <= 0 || h.active[rounds - 1]) return 0;
    int used = 1;
    for (int r = 0; r < rounds; r++)
        if (h.active[r]) used = r + 2;
    return std::min(used, rounds);
}
void note_rounds(ec_session *s, const Scalars &h, int rounds) {
    const int used = rounds_used(h, rounds);
    s->spec_rounds = used ? used + 1 : 0;
}

// extended alphabet (extended.h): links without their twin link make their components'
// walks overlap; those components are cut out of the parallel ranking (their successors saved
// in x_succ) and their dict entries listed in (component, first event) order for k_x_emulate.
// nx = the entries listed (0: every link has its twin link, nothing to do)
int x_cut(ec_session *s, unsigned int U, unsigned int &nx) {
    hipStream_t st = s->stream;
    const unsigned B = 256;
    Scalars *dsc = s->scal.as<Scalars>();
    const unsigned int N = 2 * U;
    nx = 0;
    EC_HIP(hipMemsetAsync(&dsc->nasym, 0, 16, st));  // nasym, nxl, nxs, xbad
    k_x_asym<<<grid_for(N, B), B, 0, st>>>(s->upal.as<uint8_t>(), s->succ.as<unsigned int>(), N, &dsc->nasym);
    unsigned int nasym = 0;
    EC_CHECK(d2h(s, &nasym, &dsc->nasym, 4, st));
    EC_CHECK(host_sync(s, st));
    if (kn().verbose) fprintf(stderr, "extended: %u one-way links among %u nodes\n", nasym, N);
    if (!nasym) return EC_OK;
    EC_CHECK(s->x_par.ensure((size_t)U * 4));
    EC_CHECK(s->x_irr.ensure(U));
    EC_CHECK(s->x_in.ensure(U));
    EC_CHECK(s->x_succ.ensure((size_t)N * 4));
    EC_CHECK(s->x_lk.ensure((size_t)N * 8));
    EC_CHECK(s->x_lk2.ensure((size_t)N * 8));
    EC_CHECK(s->x_lv.ensure((size_t)N * 4));
    EC_CHECK(s->x_lv2.ensure((size_t)N * 4));
    // union-find over canonical ids (CAS hooks); par then holds the roots (the tree in x_lv2)
    unsigned int *par = s->x_par.as<unsigned int>(), *tree = s->x_lv2.as<unsigned int>();
    k_x_iota<<<grid_for(U, B), B, 0, st>>>(tree, U);
    k_x_uf_link<<<grid_for(N, B), B, 0, st>>>(s->upal.as<uint8_t>(), s->succ.as<unsigned int>(), N, tree);
    k_x_uf_flatten<<<grid_for(U, B), B, 0, st>>>(U, tree, par);
    EC_HIP(hipMemsetAsync(s->x_irr.p, 0, U, st));
    k_x_mark_irr<<<grid_for(N, B), B, 0, st>>>(s->upal.as<uint8_t>(), s->succ.as<unsigned int>(), N, par,
                                              s->x_irr.as<uint8_t>());
    k_x_cut<<<grid_for(N, B), B, 0, st>>>(s->upal.as<uint8_t>(), N, par, s->x_irr.as<uint8_t>(), s->x_in.as<uint8_t>(),
                                         s->succ.as<unsigned int>(), s->x_succ.as<unsigned int>(),
                                         s->dfc.as<unsigned long long>(), s->dft.as<unsigned long long>(),
                                         s->x_lk.as<unsigned long long>(), s->x_lv.as<unsigned int>(), &dsc->nxl);
    EC_CHECK(d2h(s, &nx, &dsc->nxl, 4, st));
    EC_CHECK(host_sync(s, st));
    if (kn().verbose) fprintf(stderr, "extended: %u one-way links, %u dict entries in their components\n", nasym, nx);
    // (component, first event) order: by event, then stably by component root
    EC_CHECK(sort_pairs(s, s->x_lk.as<unsigned long long>(), s->x_lk2.as<unsigned long long>(), s->x_lv.as<unsigned int>(),
                        s->x_lv2.as<unsigned int>(), nx));
    k_x_rekey<<<grid_for(nx, B), B, 0, st>>>(s->x_lv2.as<unsigned int>(), nx, par, s->x_lk.as<unsigned long long>());
    EC_CHECK(sort_pairs(s, s->x_lk.as<unsigned long long>(), s->x_lk2.as<unsigned long long>(),
                        s->x_lv2.as<unsigned int>(), s->x_lv.as<unsigned int>(), nx));
    return EC_OK;
}

// dense ids with minimizer locality (a bucket's ids contiguous, a bucket = whole minimizers:
// the super-k-mer count, the sharded load on minimizer buckets): most links stay inside a
// rank_tile.h tile.  Hash-bucketed ids (window records, 128-bit keys, extended alphabet) have
// none -- every link would leave its tile and the contraction only add work
template <typename Index>
inline bool ids_minimizer_local(const Index &) { return false; }
template <>
inline bool ids_minimizer_local<SolidIndex>(const SolidIndex &x) { return x.sk != 0; }
template <>
inline bool ids_minimizer_local<SolidIndexW>(const SolidIndexW &x) { return x.mb != 0; }

// all_contigs:79-111 on the device from the solid set of phase_count / phase_merge
template <typename Ops, typename Index>
int phase_graph(ec_session *s, int k, unsigned int U, const Index &sidx, const unsigned int *ext_succ = nullptr) {
    hipStream_t st = s->stream;
    const unsigned B = 256;
    Scalars *dsc = s->scal.as<Scalars>();
    Scalars hsc{};
    const unsigned int N = 2 * U;
    const size_t Nn = std::max<size_t>(N, 1);
    // list ranking by tile contraction (rank_tile.h) on minimizer-local ids, the node-level
    // ruling set otherwise (EULERHIP_RANK=1 / 2 force one or the other); tile ranking needs
    // neither pred nor the node walk records
    const bool tile_rank = kn().rank == 2 || (kn().rank != 1 && ids_minimizer_local(sidx));

    // ---- links ----------------------------------------------------------------------------
    mark(s, 2 * EC_STAGE_LINKS);
    EC_CHECK(s->upal.ensure(std::max<size_t>(U, 1)));
    EC_CHECK(s->outdeg.ensure(std::max<size_t>(Nn, (Nn / 64 + 8) * 8)));  // (later: k_pred_rc's ruler bits)
    EC_CHECK(s->cand.ensure(Nn * 4));
    EC_CHECK(s->succ.ensure(Nn * 4));
    EC_CHECK(s->pred.ensure(Nn * 4));
    if (U && ext_succ) {  // partitioned links (ec_graph_finish): successors computed by the ranks
        EC_CHECK(launch_upal<Ops>(st, s->dkey.as<typename Ops::K>(), U, k, s->upal.as<uint8_t>(), &dsc->npal));
        EC_HIP(hipMemcpyAsync(s->succ.p, ext_succ, (size_t)N * 4, hipMemcpyDeviceToDevice, st));
    }
    // links by the half-edge join (join_w.h) instead of neighbour probes from ~2e6 keys on, for
    // every index (measured on the headline's minimizer index, round 4: links 0.34 ms joined
    // against 0.50 ms probed, EULERHIP_JOIN_LINKS=0)
    bool joined = false;
    const unsigned int *gate = nullptr;
    constexpr bool XT = std::is_same<Ops, OpsX>::value;  // extended alphabet (extended.h)
    if constexpr (!XT) {
        // inside the count's minimizer tables first (join_local.h), when the ids are grouped so
        if (U && !ext_succ && kn().join_links != 0 && kn().join_local != 0 &&
            (kn().join_local == 1 || kn().join_links == 1 || U >= (1u << 21)))
            EC_CHECK(links_local<Ops>(s, k, U, sidx, joined, gate));
        if (!joined && U && !ext_succ && k >= 8 && kn().join_links != 0 && (kn().join_links == 1 || U >= (1u << 21)))
        {
            if constexpr (std::is_same<Index, SolidIndexW>::value) {
                // (opt-in: config 5's junction groups overflowed the join's fixed-capacity regions,
                // sized for uniform hashes, and the probe fallback took links 39 -> 81 ms)
                if (sidx.mb && kn().join_mb == 1) EC_CHECK((links_join<Ops, JoinTM>(s, k, U, joined, gate)));
                else EC_CHECK(links_join<Ops>(s, k, U, joined, gate));
            } else {
                EC_CHECK(links_join<Ops>(s, k, U, joined, gate));
            }
        }
    }
    if (U && !ext_succ) {  // (after a join: only if it overflowed, decided on the device)
        // gated: a small grid-stride grid, so the normal case (the gate closed) costs ~2 us a
        // launch instead of one exiting block per 256 nodes
        const unsigned gn = joined ? std::min(grid_for(N, B), 2048u) : grid_for(N, B);
        k_neighbors<Ops, Index><<<gn, B, 0, st>>>(sidx, s->dkey.as<typename Ops::K>(), U, k,
                                                 s->upal.as<uint8_t>(), s->outdeg.as<uint8_t>(),
                                                 s->cand.as<unsigned int>(), joined ? nullptr : &dsc->npal, gate);
        EC_CHECK(s->nrec.ensure(Nn * sizeof(NodeRec)));
        k_succ<<<gn, B, 0, st>>>(s->upal.as<uint8_t>(), s->outdeg.as<uint8_t>(), s->cand.as<unsigned int>(), N,
                                s->succ.as<unsigned int>(), s->dfc.as<unsigned long long>(),
                                s->dft.as<unsigned long long>(), (joined || tile_rank) ? nullptr : s->nrec.as<NodeRec>(),
                                gate);
    }
    unsigned int nx = 0;  // extended alphabet: dict entries of components with one-way links
    if constexpr (XT) {
        if (U) EC_CHECK(x_cut(s, U, nx));
    }
    if (U && !tile_rank) {
        // (with the first ruler pass's counts: k_rulers_count at it = 0 below is skipped, and the
        // node records when k_succ did not write them, or wrote successors x_cut has cut since)
        EC_CHECK(s->nrec.ensure(Nn * sizeof(NodeRec)));
        EC_CHECK(s->rbc.ensure(((Nn + RULER_CHUNK - 1) / RULER_CHUNK) * 8));
        k_pred_rc<<<(unsigned int)((N + RULER_CHUNK - 1) / RULER_CHUNK), B, 0, st>>>(
            s->upal.as<uint8_t>(), s->succ.as<unsigned int>(), N, 31u, s->pred.as<unsigned int>(),
            s->rbc.as<unsigned int>(), s->dfc.as<unsigned long long>(), s->dft.as<unsigned long long>(),
            (ext_succ || joined || nx) ? s->nrec.as<NodeRec>() : nullptr, s->outdeg.as<unsigned long long>());
    }
    mark(s, 2 * EC_STAGE_LINKS + 1);

    // ---- rank (sparse ruling set + weighted Wyllie on the rulers) -------------------------
    mark(s, 2 * EC_STAGE_RANK);
    EC_CHECK(s->rid.ensure(Nn * 8));  // (ruler, offset) per node
    EC_CHECK(s->rlist.ensure(Nn * 4));
    EC_CHECK(s->rbc.ensure(((Nn + RULER_CHUNK - 1) / RULER_CHUNK) * 8));
    EC_CHECK(s->nextR.ensure(Nn * 4));
    EC_CHECK(s->st0.ensure(Nn * sizeof(RJump)));
    EC_CHECK(s->st1.ensure(Nn * sizeof(RJump)));
    EC_CHECK(s->PK.ensure(Nn * 4));
    EC_CHECK(s->RK.ensure(Nn * 4));
    EC_CHECK(s->PL.ensure(Nn * 4));
    EC_CHECK(s->PM.ensure(Nn * 8));
    unsigned int nr = 0;
    int rounds = 0;  // Wyllie rounds launched (their convergence is checked with the results)
    bool rank_async = false;     // rank_supers_async: its checks wait for the next scalar read
    const unsigned long long *async_M = nullptr;  // (the chain count on the device)
    unsigned int *async_LH = nullptr, *async_LR = nullptr;
    bool chain_paths = false;  // PK / RK of the tile ranking read through the chains (PathOf)
    s->stats.rank_rounds = 0;
    if (U && tile_rank) {
        // (1) chains of in-tile links ranked in LDS, in-tile cycles finished (rank_tile.h)
        // tiles cut at bucket starts where the count marked them (k_tile_plan), else fixed
        const bool planned = ids_minimizer_local(sidx) && s->bmark_ok;
        s->bmark_ok = false;
        // (buckets of more than ~300 keys -- config 5's 2^19 tables hold ~376 -- are cut on the
        // finer stride that may round down by up to 512: a cut inside a bucket splits nearly every
        // minimizer run of it, whose k-mers lie in hash order across the bucket's ids)
        const double per_bucket = s->stats.n_buckets ? (double)U / s->stats.n_buckets : 0.0;
        const unsigned int step = per_bucket > 300.0 ? RT_STEP_SEG : RT_STEP;
        const unsigned int ntiles = planned ? (U + step - 1) / step : (N + RT_TN - 1) / RT_TN;
        const unsigned int *tbp = nullptr;
        if (planned) {
            EC_CHECK(s->rt_tb.ensure(((size_t)ntiles + 1) * 4));
            k_tile_plan<<<grid_for(ntiles + 1ull, B), B, 0, st>>>(s->bmark.as<unsigned int>(), U, ntiles,
                                                               s->rt_tb.as<unsigned int>(), 0u, step);
            tbp = s->rt_tb.as<unsigned int>();
        }
        EC_CHECK(s->rt_tcnt.ensure(((size_t)ntiles + 1) * 8));
        EC_CHECK(s->rt_tbase.ensure(((size_t)ntiles + 1) * 8));
        EC_CHECK(s->rt_srec.ensure(Nn * sizeof(SuperRec)));
        EC_CHECK(s->rt_sidx.ensure(Nn * 4));
        EC_CHECK(s->rt_lr.ensure(Nn * 4));
        unsigned int *LH = s->pred.as<unsigned int>(), *LR = s->rt_lr.as<unsigned int>();  // (pred: free here)
        // (a planned tile keeps its chain records at its first node's offset, tb[t] - tb[0]: its
        // chains fit in its nodes, so N records suffice; fixed tiles at scratch[tile * RT_TN ..])
        EC_CHECK(s->st1.ensure(std::max<size_t>(Nn, planned ? 0 : (size_t)ntiles * RT_TN) * sizeof(RJump)));
        SuperRec *scratch = reinterpret_cast<SuperRec *>(s->st1.p);  // (dead before the Wyllie rounds)
        static_assert(sizeof(SuperRec) == sizeof(RJump), "tile scratch in the ruler state buffer");
        unsigned long long *tcnt = s->rt_tcnt.as<unsigned long long>(), *tbase = s->rt_tbase.as<unsigned long long>();
        EC_CHECK(s->rt_hasp.ensure(Nn));  // (sized here: k_tile_compact initialises it for rank_supers)
        // (2) the super list: compacted in tile order, linked, ranked by the weighted ruling set
        // (round 4 measured the same sequence as one cooperative launch: rank stage 0.63 -> 3.3
        // ms, its grid barriers far slower than the launches they replace; removed in round 5)
        unsigned int M = 0;
        rank_async = kn().rank_sync != 1;
        async_LH = LH;
        async_LR = LR;
        if (rank_async) {  // no read-back: the checks ride on the scalar read after the starts
            // the chains compacted by look-back in k_tile_chains itself (round 6: no scan, no
            // k_tile_compact, LH = super index); the status words are cleared once per allocation
            // (a reallocation is told by the capacity: the new block may come back at the old address)
            const size_t oldcap = s->rt_lb.cap;
            EC_CHECK(s->rt_lb.ensure(((size_t)ntiles + 1) * 8));
            if (s->rt_lb.cap != oldcap) {
                EC_HIP(hipMemsetAsync(s->rt_lb.p, 0, s->rt_lb.cap, st));
                s->lb_epoch = 0;
            }
            s->lb_epoch = (s->lb_epoch + 1) & ((1ull << 30) - 1);
            if (s->lb_epoch == 0) {  // (wrapped: words of 2^30 calls ago could match)
                EC_HIP(hipMemsetAsync(s->rt_lb.p, 0, s->rt_lb.cap, st));
                s->lb_epoch = 1;
            }
            TileLB lb{s->rt_lb.as<unsigned long long>(), s->lb_epoch, s->rt_srec.as<SuperRec>(),
                      s->rt_hasp.as<uint8_t>(), s->rid.as<uint2>(), &dsc->chains, &dsc->nr, &dsc->nvisited};
            async_M = &dsc->chains;
            k_tile_chains<<<ntiles, RT_NT, 0, st>>>(s->upal.as<uint8_t>(), s->succ.as<unsigned int>(), N,
                                                    s->dfc.as<unsigned long long>(), s->dft.as<unsigned long long>(),
                                                    LH, LR, tcnt, scratch, s->PK.as<unsigned int>(),
                                                    s->RK.as<unsigned int>(), s->PL.as<unsigned int>(),
                                                    s->PM.as<unsigned long long>(), 0u, tbp, lb);
            EC_CHECK(rank_supers_async(s, N, async_M, rounds, 0, LH));
            // (3) no k_expand: every reader takes a node's key and rank from its chain (PathOf)
            chain_paths = true;
        } else {
            k_tile_chains<<<ntiles, RT_NT, 0, st>>>(s->upal.as<uint8_t>(), s->succ.as<unsigned int>(), N,
                                                    s->dfc.as<unsigned long long>(), s->dft.as<unsigned long long>(),
                                                    LH, LR, tcnt, scratch, s->PK.as<unsigned int>(),
                                                    s->RK.as<unsigned int>(), s->PL.as<unsigned int>(),
                                                    s->PM.as<unsigned long long>(), 0u, tbp);
            EC_CHECK(scan_u64(s, tcnt, tbase, (size_t)ntiles + 1));
            // the chain count read back while k_tile_compact (sized by the tiles, not by M) runs:
            // the host's wake-up and next launches overlap the compaction
            unsigned long long M64 = 0;
            if (!s->rd_ev) EC_HIP(hipEventCreateWithFlags(&s->rd_ev, hipEventDisableTiming));
            EC_CHECK(d2h(s, &M64, tbase + ntiles, 8, st));
            EC_HIP(hipEventRecord(s->rd_ev, st));
            k_tile_compact<<<ntiles, 256, 0, st>>>(scratch, tcnt, tbase, s->rt_srec.as<SuperRec>(),
                                                   s->rt_sidx.as<unsigned int>(), s->rt_hasp.as<uint8_t>(),
                                                   s->rid.as<uint2>(), &dsc->nr, &dsc->nvisited, nullptr, tbp);
            EC_CHECK(host_wait(s, s->rd_ev));
            M = (unsigned int)M64;
        }
        if (!rank_async && M) {
            EC_CHECK(rank_supers(s, M, N, nr, rounds, true));
            // (3) every node: its chain's key and rank + its offset in the chain
            k_expand<<<grid_for(N, B), B, 0, st>>>(LH, LR, N, s->rt_sidx.as<unsigned int>(), s->rt_pks.as<unsigned int>(),
                                                  s->rt_rks.as<unsigned int>(), s->PK.as<unsigned int>(),
                                                  s->RK.as<unsigned int>());
        }
    }
    if (U && !tile_rank) {
        EC_HIP(hipMemsetAsync(s->rid.p, 0xFF, Nn * 8, st));
        EC_CHECK(s->nrec.ensure(Nn * sizeof(NodeRec)));
        unsigned int masks[4] = {31u, 7u, 1u, 0u};
        unsigned int r0 = 0;
        for (int it = 0; it < 4; it++) {
            const unsigned int nblk = (unsigned int)((N + RULER_CHUNK - 1) / RULER_CHUNK);
            if (it)  // (it = 0: counted by k_pred_rc with masks[0])
                k_rulers_count<<<nblk, B, 0, st>>>(s->upal.as<uint8_t>(), s->pred.as<unsigned int>(), N, masks[it],
                                                   it == 0, s->rid.as<uint2>(), s->rbc.as<unsigned int>());
            EC_CHECK(scan_incl_u32(s, s->rbc.as<unsigned int>(), s->rbc.as<unsigned int>() + nblk, nblk));
            k_rulers<<<nblk, B, 0, st>>>(s->upal.as<uint8_t>(), s->pred.as<unsigned int>(), N, masks[it], it == 0,
                                         s->rbc.as<unsigned int>() + nblk, &dsc->nr, s->rid.as<uint2>(),
                                         s->rlist.as<unsigned int>(),
                                         it == 0 ? s->outdeg.as<unsigned long long>() : nullptr);
            k_rulers_total<<<1, 1, 0, st>>>(s->rbc.as<unsigned int>() + nblk, nblk, &dsc->nr);
            k_walk<<<2048, B, 0, st>>>(s->nrec.as<NodeRec>(), s->rlist.as<unsigned int>(), r0, &dsc->nr,
                                      masks[it], s->rid.as<uint2>(),
                                      s->nextR.as<unsigned int>(), s->st0.as<RJump>(), &dsc->nvisited);
            EC_CHECK(d2h(s, &hsc, dsc, sizeof(Scalars), st));
            EC_CHECK(host_sync(s, st));
            r0 = hsc.nr;
            if (hsc.nvisited + hsc.npal >= N) break;
        }
        nr = hsc.nr;
        if (hsc.nvisited + hsc.npal != N) {
            set_error("ruling set covered %llu of %u nodes", (unsigned long long)(hsc.nvisited + hsc.npal), N);
                return EC_ERR_STATE;
        }
        k_rjump_init<<<grid_for(nr, B), B, 0, st>>>(s->nextR.as<unsigned int>(), nr, s->st0.as<RJump>());
        rounds = 1;
        while ((1ull << (rounds - 1)) < (unsigned long long)nr) rounds++;
        rounds = std::min(rounds + 1, 63);
        RJump *bufs[2] = {s->st0.as<RJump>(), s->st1.as<RJump>()};
        for (int r = 0; r < rounds; r++)
            k_rjump<<<grid_for(nr, B), B, 0, st>>>(bufs[r & 1], bufs[(r + 1) & 1], nr, N,
                                                  r ? &dsc->active[r - 1] : nullptr, &dsc->active[r],
                                                  &dsc->final_sel, (unsigned)((r + 1) & 1));
        k_finalize<<<grid_for(N, B), B, 0, st>>>(s->upal.as<uint8_t>(), s->succ.as<unsigned int>(),
                                                s->rid.as<uint2>(), s->rlist.as<unsigned int>(), bufs[0], bufs[1],
                                                &dsc->final_sel, &dsc->active[rounds - 1], N, s->PK.as<unsigned int>(),
                                                s->RK.as<unsigned int>(), s->PL.as<unsigned int>(),
                                                s->PM.as<unsigned long long>());
        k_cycle_len<<<grid_for(nr, B), B, 0, st>>>(s->nextR.as<unsigned int>(), s->rlist.as<unsigned int>(), bufs[0],
                                                  bufs[1], &dsc->final_sel, &dsc->active[rounds - 1], nr,
                                                  s->PL.as<unsigned int>(),
                                                  s->PM.as<unsigned long long>());
    }
    s->stats.n_rulers = nr;
    mark(s, 2 * EC_STAGE_RANK + 1);

    // ---- starts + order -------------------------------------------------------------------
    const PathOf P = chain_paths ? PathOf{s->PK.as<unsigned int>(), s->RK.as<unsigned int>(), async_LH, async_LR,
                                          s->rt_pks.as<unsigned int>(), s->rt_rks.as<unsigned int>()}
                                 : path_of(s->PK.as<unsigned int>(), s->RK.as<unsigned int>());
    mark(s, 2 * EC_STAGE_STARTS);
    EC_CHECK(s->cidxOf.ensure(Nn * 4));
    EC_CHECK(s->skeys.ensure(Nn * 8));
    EC_CHECK(s->svals.ensure(Nn * 4));
    EC_CHECK(s->skeys2.ensure(Nn * 8));
    EC_CHECK(s->svals2.ensure(Nn * 4));
    // the emission's node maps, cleared before the starts' read-back (the device works through
    // them while the host waits)
    EC_CHECK(s->headOf.ensure(Nn * 4));
    EC_CHECK(s->tailOf.ensure(Nn * 4));
    EC_HIP(hipMemsetAsync(s->headOf.p, 0xFF, Nn * 4, st));
    EC_HIP(hipMemsetAsync(s->tailOf.p, 0xFF, Nn * 4, st));
    EC_HIP(hipMemsetAsync(&dsc->skew, 0, 4, st));  // k_emit: a position past the character bound
    unsigned long long async_M64 = 0;
    auto starts_pass = [&]() -> int {
    EC_HIP(hipMemsetAsync(s->cidxOf.p, 0xFF, Nn * 4, st));
    if (U)
    {
        const unsigned int nblk = (unsigned int)((N + RULER_CHUNK - 1) / RULER_CHUNK);
        unsigned int *bc = s->rbc.as<unsigned int>(), *bs = bc + nblk;
        // the start bits between the two passes live in `cand` (free after the links)
        EC_CHECK(s->cand.ensure(std::max<size_t>(Nn * 4, (Nn / 64 + 8) * 8)));
        unsigned long long *smask = s->cand.as<unsigned long long>();
        k_starts_count<<<nblk, B, 0, st>>>(s->upal.as<uint8_t>(), s->dfc.as<unsigned long long>(),
                                           s->dft.as<unsigned long long>(), P,
                                           s->PM.as<unsigned long long>(), N, bc, smask,
                                           nx ? s->x_in.as<uint8_t>() : nullptr);
        EC_CHECK(scan_incl_u32(s, bc, bs, nblk));
        k_starts_write<<<nblk, B, 0, st>>>(s->upal.as<uint8_t>(), s->dfc.as<unsigned long long>(),
                                           s->dft.as<unsigned long long>(), P,
                                           s->PM.as<unsigned long long>(), N, bs, smask,
                                           s->skeys.as<unsigned long long>(), s->svals.as<unsigned int>(), 0u,
                                           &dsc->nstarts);
    }
    EC_CHECK(d2h(s, &hsc, dsc, sizeof(Scalars), st));  // nstarts, active[], the chain count
    EC_CHECK(host_sync(s, st));
    async_M64 = hsc.chains;
    return EC_OK;
    };
    EC_CHECK(starts_pass());
    if (rank_async) {
        const unsigned int Ma = (unsigned int)async_M64;
        nr = hsc.nr;
        s->stats.n_rulers = nr;
        if (kn().verbose)
            fprintf(stderr, "rank: %u oriented nodes, %u chains (tile contraction), %u rulers, %llu visited\n", N, Ma,
                    nr, (unsigned long long)hsc.nvisited);
        if (Ma) note_rounds(s, hsc, rounds);
        if (hsc.nvisited != Ma || (Ma && hsc.active[rounds - 1] != 0)) {
            // a cycle of chains no ruler reached (or unconverged rounds): the ranking with its
            // host-checked ruler passes, then the starts again
            if (kn().verbose)
                fprintf(stderr, "rank: one ruler pass covered %llu of %u chains, ranking again\n",
                        (unsigned long long)hsc.nvisited, Ma);
            rank_async = false;
            // (the look-back compaction's LH: super index per node, at heads the head -> index map)
            EC_CHECK(rank_supers(s, Ma, N, nr, rounds, false, async_LH));  // (PathOf reads the new PKs / RKs)
            s->stats.n_rulers = nr;
            EC_CHECK(starts_pass());
        }
    }
    if (rounds) {
        unsigned int used = 1;
        for (int r = 0; r < rounds; r++)
            if (hsc.active[r]) used = r + 2;
        s->stats.rank_rounds = std::min<unsigned int>(used, rounds);
        if (hsc.active[rounds - 1] != 0) {
            set_error("ruler list ranking did not converge in %d rounds", rounds);
            return EC_ERR_STATE;
        }
    }
    unsigned int nc = hsc.nstarts;
    unsigned int nsort = nc;
    if (nx) {  // all_contigs on the components with one-way links, their starts after the others
        EC_CHECK(s->x_done.ensure(Nn));
        EC_CHECK(s->x_len.ensure((size_t)nx * 4));
        EC_CHECK(s->x_m.ensure((size_t)nx * 4));
        EC_CHECK(s->x_cid.ensure((size_t)nx * 4));
        EC_HIP(hipMemsetAsync(s->x_done.p, 0, Nn, st));
        k_x_emulate<<<grid_for(nx, 64), 64, 0, st>>>(
            s->x_lv.as<unsigned int>(), nx, s->x_par.as<unsigned int>(), s->upal.as<uint8_t>(),
            s->x_succ.as<unsigned int>(), s->dkey.as<K128>(), k, N, s->dfc.as<unsigned long long>(),
            s->dft.as<unsigned long long>(), s->x_done.as<uint8_t>(), s->skeys.as<unsigned long long>() + nc,
            s->svals.as<unsigned int>() + nc, s->x_len.as<unsigned int>(), s->x_m.as<unsigned int>(), &dsc->nxs,
            &dsc->xbad);
        unsigned int xs[2] = {0, 0};
        EC_CHECK(d2h(s, xs, &dsc->nxs, 8, st));
        EC_CHECK(host_sync(s, st));
        if (xs[1]) {
            set_error("a contig walk enters a cycle without its start: the reference's get_contig_forward "
                      "(referenceAssembler.py:59-77) never returns on this input");
            return EC_ERR_STATE;
        }
        nsort = nc + nx;  // (the emulation's non-starts carry key NONE: sorted past the starts)
        nc += xs[0];
    }
    s->stats.n_contigs = nc;
    EC_CHECK(s->cwalk.ensure((size_t)std::max(nc, 1u) * sizeof(Walk)));
    EC_CHECK(s->coff.ensure((size_t)(nc + 1) * 8));
    EC_CHECK(s->ewalk.ensure((size_t)std::max(nc, 1u) * sizeof(EWalk)));
    // few starts: order, walks, offsets and emission records in one workgroup (k_starts_small)
    const bool small = !nx && nc && nc <= SMALL_STARTS && !kn().no_small_starts;
    if (small)
        k_starts_small<<<1, SMALL_STARTS_NT, 0, st>>>(
            s->skeys.as<unsigned long long>(), s->svals.as<unsigned int>(), nc, s->upal.as<uint8_t>(),
            P, s->PL.as<unsigned int>(), k,
            s->svals2.as<unsigned int>(), s->cidxOf.as<unsigned int>(), s->coff.as<unsigned long long>(),
            s->cwalk.as<Walk>(), s->ewalk.as<EWalk>());
    if (nsort && !small)
        EC_CHECK(sort_pairs(s, s->skeys.as<unsigned long long>(), s->skeys2.as<unsigned long long>(),
                            s->svals.as<unsigned int>(), s->svals2.as<unsigned int>(), nsort));
    const unsigned int *sorted_nodes = s->svals2.as<unsigned int>();
    if (!small) {
    EC_CHECK(s->clen.ensure((size_t)(nc + 1) * 8));
    EC_HIP(hipMemsetAsync(s->clen.p, 0, (size_t)(nc + 1) * 8, st));
    if (nc) {
        k_contig_len<<<grid_for(nc, B), B, 0, st>>>(s->upal.as<uint8_t>(), P, s->PL.as<unsigned int>(), sorted_nodes, nc,
                                                   k, s->cidxOf.as<unsigned int>(), s->clen.as<unsigned long long>(),
                                                   s->cwalk.as<Walk>(), nx ? s->x_len.as<unsigned int>() : nullptr,
                                                   nx ? s->x_cid.as<unsigned int>() : nullptr);
    }
    EC_CHECK(scan_u64(s, s->clen.as<unsigned long long>(), s->coff.as<unsigned long long>(), nc + 1));
    }
    // the total travels with the other results (no round trip here): the character buffer is
    // sized for the bound 2U + nc (k - 1) (a walk covers at most its path; a self-twin path's
    // nodes are up to twice its canonical k-mers)
    EC_CHECK(s->h_coff.resize(nc + 1));
    EC_CHECK(d2h(s, &s->h_coff[nc], s->coff.as<unsigned long long>() + nc, 8, st));
    // the results' copies to host memory run on the output stream, each as soon as its data is
    // final: the contig offsets here (overlapping emission and GFA), the characters after the
    // emission, the link offsets after the GFA counts (ecoli10m_err: 1.1 M contigs, 47 MB of
    // results copied after GFA took ~1 ms in line)
    auto ostream_ready = [&]() -> int {
        if (!s->ostream) EC_HIP(hipStreamCreateWithFlags(&s->ostream, hipStreamNonBlocking));
        for (auto &e : s->oev)
            if (!e) EC_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        return EC_OK;
    };
    // (only for many contigs: the event / stream-wait / copy calls cost the host ~30 us, more
    // than the headline's few bytes of offsets and link counts take in line)
    const bool ocopy = nc >= OCOPY_MIN;
    EC_CHECK(ostream_ready());
    if (ocopy) {
        EC_HIP(hipEventRecord(s->oev[2], st));
        EC_HIP(hipStreamWaitEvent(s->ostream, s->oev[2], 0));
        EC_HIP(hipMemcpyAsync(s->h_coff.data(), s->coff.p, (size_t)nc * 8, hipMemcpyDeviceToHost, s->ostream));
    }
    mark(s, 2 * EC_STAGE_STARTS + 1);
    uint64_t chars_bound = 2ull * U + (uint64_t)nc * (uint64_t)(k - 1);
    if (nx) {  // emulated contigs may overlap: the bound is their exact total
        unsigned long long tot = 0;
        EC_CHECK(d2h(s, &tot, s->coff.as<unsigned long long>() + nc, 8, st));
        EC_CHECK(host_sync(s, st));
        chars_bound = std::max<uint64_t>(chars_bound, tot);
    }

    // ---- emit -----------------------------------------------------------------------------
    mark(s, 2 * EC_STAGE_EMIT);
    EC_CHECK(s->chars.ensure(std::max<size_t>(chars_bound, 1) + 16));  // (+16: k_pack_chars reads 16 at a time)
    EC_CHECK(s->cfirst.ensure((size_t)std::max(nc, 1u) * 4));
    EC_CHECK(s->clast.ensure((size_t)std::max(nc, 1u) * 4));
    if (nc && !small)
        k_ewalk<<<grid_for(nc, B), B, 0, st>>>(s->cwalk.as<Walk>(), s->coff.as<unsigned long long>(), nc,
                                              s->ewalk.as<EWalk>());
    if (U)
        k_emit<Ops><<<grid_for(N, B), B, 0, st>>>(s->upal.as<uint8_t>(), P,
                                            s->PL.as<unsigned int>(), s->dkey.as<typename Ops::K>(),
                                            s->cidxOf.as<unsigned int>(), s->ewalk.as<EWalk>(),
                                            N, k, s->chars.as<char>(), std::max<uint64_t>(chars_bound, 1),
                                            s->cfirst.as<unsigned int>(), s->clast.as<unsigned int>(),
                                            s->headOf.as<unsigned int>(), s->tailOf.as<unsigned int>(), &dsc->skew);
    if constexpr (XT) {
        if (nx) {
            EC_CHECK(s->x_head.ensure(Nn * 4));
            EC_CHECK(s->x_tail.ensure(Nn * 4));
            EC_HIP(hipMemsetAsync(s->x_head.p, 0, Nn * 4, st));
            EC_HIP(hipMemsetAsync(s->x_tail.p, 0, Nn * 4, st));
            k_x_emit<<<grid_for(nx, B), B, 0, st>>>(
                s->x_lv.as<unsigned int>(), s->x_len.as<unsigned int>(), s->x_m.as<unsigned int>(),
                s->x_cid.as<unsigned int>(), s->skeys.as<unsigned long long>() + hsc.nstarts, nx, s->upal.as<uint8_t>(),
                s->x_succ.as<unsigned int>(), s->dkey.as<K128>(), k, s->coff.as<unsigned long long>(),
                s->chars.as<char>(), s->cfirst.as<unsigned int>(), s->clast.as<unsigned int>(),
                s->x_head.as<unsigned int>(), s->x_tail.as<unsigned int>());
            k_x_heads<<<grid_for(N, B), B, 0, st>>>(N, s->x_head.as<unsigned int>(), s->x_tail.as<unsigned int>(),
                                                    s->headOf.as<unsigned int>(), s->tailOf.as<unsigned int>());
        }
    }
    // the characters' copy to host memory starts on the output stream as soon as the emission is
    // done, sized by the previous call's total (a stream of equal batches, the bench's steps): it
    // overlaps GFA and the link compaction instead of following a read-back of the total; a
    // larger total is copied again in full after the read-back
    // standard alphabet: the characters travel as 2-bit codes (a quarter of the PCIe bytes)
    const bool pack = !XT && kn().no_char_pack == 0;
    const void *csrc = s->chars.p;
    if (pack) {
        const uint64_t cap16 = (std::max<uint64_t>(chars_bound, 1) + 15) / 16;
        EC_CHECK(s->dchars.ensure(cap16 * 4));
        k_pack_chars<<<std::min(grid_for(cap16, B), 8192u), B, 0, st>>>(
            s->chars.as<uint4>(), s->coff.as<unsigned long long>() + nc, cap16, s->dchars.as<uint32_t>());
        csrc = s->dchars.p;
    }
    auto hbytes = [&](uint64_t n) { return pack ? (n + 3) / 4 : n; };  // host bytes of n characters
    uint64_t pre = 0;
    if (s->last_nchars && s->last_nchars <= chars_bound && kn().no_spec == 0) {
        pre = s->last_nchars;
        EC_CHECK(s->h_chars.resize(hbytes(pre)));
        EC_HIP(hipEventRecord(s->oev[0], st));
        EC_HIP(hipStreamWaitEvent(s->ostream, s->oev[0], 0));
        EC_HIP(hipMemcpyAsync(s->h_chars.data(), csrc, hbytes(pre), hipMemcpyDeviceToHost, s->ostream));
        EC_HIP(hipEventRecord(s->oev[1], s->ostream));
    }
    s->last_nchars = 0;
    mark(s, 2 * EC_STAGE_EMIT + 1);

    // ---- GFA ------------------------------------------------------------------------------
    mark(s, 2 * EC_STAGE_GFA);
    EC_CHECK(s->lk.ensure((size_t)std::max(nc, 1u) * 16 * 8));
    EC_CHECK(s->lcnt.ensure((size_t)std::max(nc, 1u) * 2 * 4));
    if (nc)
        k_gfa<Ops, Index><<<grid_for(nc, B), B, 0, st>>>(sidx, s->dkey.as<typename Ops::K>(),
                                            s->upal.as<uint8_t>(), s->cfirst.as<unsigned int>(),
                                            s->clast.as<unsigned int>(), s->headOf.as<unsigned int>(),
                                            s->tailOf.as<unsigned int>(), nc, k, s->lk.as<long long>(),
                                            s->lcnt.as<unsigned int>());
    mark(s, 2 * EC_STAGE_GFA + 1);

    // ---- results to host (links compacted on the device: only the used entries travel) -----
    const unsigned int n2 = 2 * nc;
    s->links_compact = true;
    EC_CHECK(s->h_lc8.resize(n2));
    if (!nc) s->h_coff[0] = 0;
    if (nc && !ocopy) EC_CHECK(d2h(s, s->h_coff.data(), s->coff.p, (size_t)nc * 8, st));
    unsigned long long nlinks64 = 0;
    if (nc && small) {
        // (n2 <= 8192: counts, offsets and the compacted links in one launch; the links' bound
        // 8 n2 travels with the total, so no second round trip follows)
        EC_CHECK(s->lc8.ensure(n2));
        EC_CHECK(s->dcounts.ensure((size_t)n2 * 8 * 4));
        EC_CHECK(s->skeys2.ensure(8));
        k_links_small<<<1, SMALL_LINK_NT, 0, st>>>(s->lk.as<long long>(), s->lcnt.as<unsigned int>(), n2,
                                                   s->lc8.as<uint8_t>(), s->dcounts.as<uint32_t>(),
                                                   s->skeys2.as<unsigned long long>());
        EC_CHECK(d2h(s, s->h_lc8.data(), s->lc8.p, n2, st));
        EC_CHECK(s->h_links32.resize((size_t)n2 * 8));
        EC_CHECK(d2h(s, s->h_links32.data(), s->dcounts.p, (size_t)n2 * 8 * 4, st));
        EC_CHECK(d2h(s, &nlinks64, s->skeys2.p, 8, st));
    } else if (nc) {
        EC_CHECK(s->skeys.ensure(((size_t)n2 + 1) * 8));   // per-side counts as u64 (starts sorted)
        EC_CHECK(s->skeys2.ensure(((size_t)n2 + 1) * 8));  // their exclusive scan = link offsets
        // (the counts as bytes in a buffer of their own: the scan's temporary storage is s->tmp)
        EC_CHECK(s->lc8.ensure(n2));
        k_lcnt64<<<grid_for(n2 + 1ull, B), B, 0, st>>>(s->lcnt.as<unsigned int>(), n2, s->skeys.as<unsigned long long>(),
                                                       s->lc8.as<uint8_t>());
        if (ocopy) {
            EC_HIP(hipEventRecord(s->oev[3], st));
            EC_HIP(hipStreamWaitEvent(s->ostream, s->oev[3], 0));
            EC_HIP(hipMemcpyAsync(s->h_lc8.data(), s->lc8.p, n2, hipMemcpyDeviceToHost, s->ostream));
        } else {
            EC_CHECK(d2h(s, s->h_lc8.data(), s->lc8.p, n2, st));
        }
        EC_CHECK(scan_u64(s, s->skeys.as<unsigned long long>(), s->skeys2.as<unsigned long long>(), (size_t)n2 + 1));
        EC_CHECK(d2h(s, &nlinks64, s->skeys2.as<unsigned long long>() + n2, 8, st));
    }
    unsigned int emit_bad = 0;
    EC_CHECK(d2h(s, &emit_bad, &dsc->skew, 4, st));
    EC_CHECK(host_sync(s, st));  // h_coff[nc] (the characters), the link total
    const uint64_t nchars = s->h_coff[nc];
    if (emit_bad || nchars > chars_bound) EC_HIP(hipStreamSynchronize(s->ostream));  // (no copy left in flight)
    if (emit_bad) {
        set_error("contig characters past their bound %llu (inconsistent ranking)", (unsigned long long)chars_bound);
        return EC_ERR_STATE;
    }
    s->stats.n_contig_chars = nchars;
    if (nchars > chars_bound) {
        set_error("contig characters %llu past their bound %llu", (unsigned long long)nchars,
                  (unsigned long long)chars_bound);
        return EC_ERR_STATE;
    }
    if (pre && nchars > pre) EC_HIP(hipEventSynchronize(s->oev[1]));  // (before h_chars may move)
    EC_CHECK(s->h_chars.resize(hbytes(nchars)));
    s->chars_packed = pack;
    s->nchars_host = nchars;
    bool again = nchars > pre;  // (a second round trip: characters or links still to copy)
    if (nchars > pre) EC_CHECK(d2h(s, s->h_chars.data(), csrc, hbytes(nchars), st));
    const uint64_t nlinks = nlinks64;
    EC_CHECK(s->h_links32.resize(nlinks));  // (small: the copied bound's first nlinks stay)
    if (nlinks && !small) {
        again = true;
        EC_CHECK(s->dcounts.ensure(nlinks * 4));
        k_links_compact<uint32_t><<<grid_for(n2, B), B, 0, st>>>(s->lk.as<long long>(), s->lcnt.as<unsigned int>(),
                                                                s->skeys2.as<unsigned long long>(), n2,
                                                                s->dcounts.as<uint32_t>());
        EC_CHECK(d2h(s, s->h_links32.data(), s->dcounts.p, nlinks * 4, st));
    }
    if (again) EC_CHECK(host_sync(s, st));
    if (ocopy || pre) EC_HIP(hipStreamSynchronize(s->ostream));  // (offsets, characters, link counts)
    s->last_nchars = nchars;
    s->stats.n_links = nlinks;

    s->stats.n_dict = 2ull * U - hsc.npal;  // len(build()): palindromes have one entry

    collect_timing(s);
    s->have = true;
    s->stats_ok = true;
    return EC_OK;
}

// ---- multi-GPU partitioned finish (distributed.py): each rank ranks and emits its own segment --
// of the loaded (gathered) solid set, canonical ids [lo, hi) = oriented nodes [n0, n1):
//   ec_graph_chains_part  its links' chains ranked in LDS (rank_tile.h) -> its super records
//   ec_graph_rank_supers  every rank: the job's super list (all-gathered, rank order) ranked
//   ec_graph_starts_part  its nodes' keys / ranks, its contig starts -> start records
//   ec_graph_layout       every rank: the job's starts (all-gathered) in event order, offsets
//   ec_graph_emit_part    its nodes' characters at their global positions, its contig ends
//   ec_graph_collect      rank 0: the summed characters / ends -> GFA links and the results
// the chain records of k_tile_chains compacted into d_super (M of them)
int part_chains_copy(ec_session *s, uint64_t M, unsigned int ntiles, bool planned, SuperRec *d_super) {
    hipStream_t st = s->stream;
    if (M)
        k_tile_compact<<<ntiles, 256, 0, st>>>(s->chain_scr, s->rt_tcnt.as<unsigned long long>(),
                                               s->rt_tbase.as<unsigned long long>(), d_super,
                                               s->rt_sidx.as<unsigned int>(), nullptr, nullptr, nullptr, nullptr,
                                               nullptr, planned ? s->rt_tb.as<unsigned int>() : nullptr);
    EC_CHECK(host_sync(s, st));
    return EC_OK;
}

template <typename Ops>
int part_chains(ec_session *s, uint64_t lo, uint64_t hi, const uint32_t *d_succ, SuperRec *d_super,
                uint64_t *n_super) {
    hipStream_t st = s->stream;
    const unsigned B = 256;
    Scalars *dsc = s->scal.as<Scalars>();
    const unsigned int U = (unsigned int)s->n_dense, N = 2 * U;
    const size_t Nn = std::max<size_t>(N, 1);
    const unsigned int n0 = (unsigned int)(2 * lo), n1 = (unsigned int)(2 * hi);
    EC_CHECK(s->upal.ensure(std::max<size_t>(U, 1)));
    EC_CHECK(s->succ.ensure(Nn * 4));
    EC_CHECK(s->PK.ensure(Nn * 4));
    EC_CHECK(s->RK.ensure(Nn * 4));
    EC_CHECK(s->PL.ensure(Nn * 4));
    EC_CHECK(s->PM.ensure(Nn * 8));
    EC_CHECK(s->pred.ensure(Nn * 4));
    EC_CHECK(s->rt_lr.ensure(Nn * 4));
    EC_CHECK(s->rt_sidx.ensure(Nn * 4));
    if (!s->placed) {  // (a placed segment has its flags and links already: ec_graph_place / join)
        EC_HIP(hipMemsetAsync(&dsc->npal, 0, 4, st));
        EC_CHECK(launch_upal<Ops>(st, s->dkey.as<typename Ops::K>(), U, s->k, s->upal.as<uint8_t>(), &dsc->npal));
    }
    if (n1 > n0 && d_succ)
        EC_HIP(hipMemcpyAsync(s->succ.as<unsigned int>() + n0, d_succ, (size_t)(n1 - n0) * 4, hipMemcpyDeviceToDevice,
                              st));
    // tiles cut at the bucket starts this rank's owner merge marked (its output is this segment)
    const bool planned = s->seg_marks && s->seg_marks == hi - lo && hi > lo;
    const unsigned int ntiles =
        planned ? (unsigned int)((hi - lo + RT_STEP_SEG - 1) / RT_STEP_SEG) : (n1 - n0 + RT_TN - 1) / RT_TN;
    const unsigned int *tbp = nullptr;
    if (planned) {
        EC_CHECK(s->rt_tb.ensure(((size_t)ntiles + 1) * 4));
        k_tile_plan<<<grid_for(ntiles + 1ull, B), B, 0, st>>>(s->bmark.as<unsigned int>(), (unsigned int)(hi - lo),
                                                           ntiles, s->rt_tb.as<unsigned int>(), (unsigned int)lo,
                                                           RT_STEP_SEG);
        tbp = s->rt_tb.as<unsigned int>();
    }
    EC_CHECK(s->rt_tcnt.ensure(((size_t)ntiles + 1) * 8));
    EC_CHECK(s->rt_tbase.ensure(((size_t)ntiles + 1) * 8));
    // (planned tiles keep their chain records at node offsets: 2 (hi - lo) records.)  A placed
    // segment's junction slots (4 a key of >= 16 B: >= the 64 B a key of chain records) are free
    // once ec_graph_place_copy gathered them, so the records go there instead of a buffer of
    // their own (12.6 GB at one config-5 rank); the pending place records are dropped with them
    const size_t scr_bytes =
        std::max<size_t>(planned ? 2 * (size_t)(hi - lo) : (size_t)ntiles * RT_TN, 1) * sizeof(SuperRec);
    DevBuf &scr = s->placed && s->jrec.cap >= scr_bytes ? s->jrec : s->st1;
    if (&scr == &s->jrec && s->hold.kind == 1) s->hold.kind = 0;
    EC_CHECK(scr.ensure(scr_bytes));
    unsigned long long *tcnt = s->rt_tcnt.as<unsigned long long>(), *tbase = s->rt_tbase.as<unsigned long long>();
    SuperRec *scratch = reinterpret_cast<SuperRec *>(scr.p);
    s->chain_scr = scratch;
    if (!ntiles) EC_HIP(hipMemsetAsync(tcnt, 0, 8, st));  // (k_tile_chains zeroes tcnt[ntiles])
    if (ntiles)
        k_tile_chains<<<ntiles, RT_NT, 0, st>>>(s->upal.as<uint8_t>(), s->succ.as<unsigned int>(), n1,
                                                s->dfc.as<unsigned long long>(), s->dft.as<unsigned long long>(),
                                                s->pred.as<unsigned int>(), s->rt_lr.as<unsigned int>(), tcnt, scratch,
                                                s->PK.as<unsigned int>(), s->RK.as<unsigned int>(),
                                                s->PL.as<unsigned int>(), s->PM.as<unsigned long long>(), n0, tbp);
    EC_CHECK(scan_u64(s, tcnt, tbase, (size_t)ntiles + 1));
    unsigned long long M = 0;
    EC_CHECK(d2h(s, &M, tbase + ntiles, 8, st));
    EC_CHECK(host_sync(s, st));
    *n_super = M;
    s->seg_n0 = n0;
    s->seg_n1 = n1;
    if (!d_super) {  // counted only: ec_graph_chains_copy compacts them
        s->hold = ec_session::Pending{2, M, ntiles, planned};
        return EC_OK;
    }
    return part_chains_copy(s, M, ntiles, planned, d_super);
}

int part_rank(ec_session *s, const SuperRec *d_all, uint64_t M) {
    hipStream_t st = s->stream;
    s->hold.kind = 0;  // (the next steps reuse the held records' buffers)
    Scalars *dsc = s->scal.as<Scalars>();
    const unsigned int N = 2 * (unsigned int)s->n_dense;
    s->stats.n_rulers = 0;
    if (!M) return EC_OK;
    // the super list's buffers sized by its chain count (1/16 spare on first allocation, so a
    // step whose count is a little above the last one's reuses them), not by the node count:
    // config 5's one-rank step ranks 21 M chains of 400 M nodes, where node-sized ruler state
    // held ~38 GB (r06_h)
    const size_t mc = (size_t)M + 4096;
    EC_CHECK(s->rt_srec.ensure(mc * sizeof(SuperRec), 16));
    EC_HIP(hipMemcpyAsync(s->rt_srec.p, d_all, (size_t)M * sizeof(SuperRec), hipMemcpyDeviceToDevice, st));
    k_super_index<<<grid_for(M, 256), 256, 0, st>>>(s->rt_srec.as<SuperRec>(), (unsigned int)M,
                                                    s->rt_sidx.as<unsigned int>());
    unsigned int nr = 0;
    int rounds = 0;
    if (kn().rank_sync != 1) {
        // rank_supers_async (one read-back at the end instead of one per ruler pass plus the
        // launch backlog after it): M on the device, the ruler state initialised here
        EC_CHECK(s->rt_hasp.ensure(mc, 16));
        EC_CHECK(s->rid.ensure(mc * 8, 16));
        EC_CHECK(s->st0.ensure(mc * sizeof(RJump), 16));
        EC_CHECK(s->st1.ensure(mc * sizeof(RJump), 16));
        EC_CHECK(s->rt_tbase.ensure(8));
        // the chain count on the device, the ruler state initialised: one launch (six memsets
        // cost ~40 us of launch gaps)
        k_part_rank_init<<<std::min(grid_for(M, 256), 2048u), 256, 0, st>>>(
            s->rt_tbase.as<unsigned long long>(), (unsigned int)M, s->rt_hasp.as<uint8_t>(), s->rid.as<uint2>(), &dsc->nr,
            &dsc->nvisited);
        EC_CHECK(rank_supers_async(s, N, s->rt_tbase.as<unsigned long long>(), rounds, (unsigned int)M));
        Scalars hsc{};
        EC_CHECK(d2h(s, &hsc, dsc, sizeof(Scalars), st));
        EC_CHECK(host_sync(s, st));
        note_rounds(s, hsc, rounds);
        if (hsc.nvisited == M && hsc.active[rounds - 1] == 0) {
            s->stats.n_rulers = hsc.nr;
            s->stats.rank_rounds = rounds_used(hsc, rounds);
            return EC_OK;
        }
        if (kn().verbose)
            fprintf(stderr, "part_rank: one ruler pass covered %llu of %llu chains, ranking again\n",
                    (unsigned long long)hsc.nvisited, (unsigned long long)M);
    }
    EC_CHECK(rank_supers(s, (unsigned int)M, N, nr, rounds));
    s->stats.n_rulers = nr;
    unsigned int act = 0;
    EC_CHECK(d2h(s, &act, &dsc->active[rounds - 1], 4, st));
    EC_CHECK(host_sync(s, st));
    if (act) {
        set_error("chain list ranking did not converge in %d rounds", rounds);
        return EC_ERR_STATE;
    }
    s->stats.rank_rounds = rounds;
    return EC_OK;
}

// the start records of the nodes k_starts_write listed (cnt of them) into d_starts
int part_starts_copy(ec_session *s, uint64_t cnt, StartRec *d_starts) {
    hipStream_t st = s->stream;
    if (cnt)
        k_start_recs<<<grid_for(cnt, 256), 256, 0, st>>>(s->svals.as<unsigned int>(), (unsigned int)cnt,
                                                         s->upal.as<uint8_t>(), s->dfc.as<unsigned long long>(),
                                                         s->dft.as<unsigned long long>(),
                                                         path_of(s->PK.as<unsigned int>(), s->RK.as<unsigned int>()),
                                                         s->PL.as<unsigned int>(), s->k, d_starts);
    EC_CHECK(host_sync(s, st));
    return EC_OK;
}

int part_starts(ec_session *s, bool have_supers, StartRec *d_starts, uint64_t *n_starts) {
    hipStream_t st = s->stream;
    const unsigned B = 256;
    const unsigned int n0 = (unsigned int)s->seg_n0, n1 = (unsigned int)s->seg_n1;
    const size_t Nn = std::max<size_t>(2 * (size_t)s->n_dense, 1);
    *n_starts = 0;
    if (n1 <= n0) return EC_OK;
    if (have_supers)
        k_expand<<<grid_for(n1 - n0, B), B, 0, st>>>(s->pred.as<unsigned int>(), s->rt_lr.as<unsigned int>(), n1,
                                                     s->rt_sidx.as<unsigned int>(), s->rt_pks.as<unsigned int>(),
                                                     s->rt_rks.as<unsigned int>(), s->PK.as<unsigned int>(),
                                                     s->RK.as<unsigned int>(), n0);
    const unsigned int nblk = (n1 - n0 + RULER_CHUNK - 1) / RULER_CHUNK;
    EC_CHECK(s->rbc.ensure((size_t)nblk * 8 + 8));
    EC_CHECK(s->cand.ensure(((size_t)(n1 - n0) / 64 + 8) * 8));
    EC_CHECK(s->skeys.ensure(Nn * 8));
    EC_CHECK(s->svals.ensure(Nn * 4));
    unsigned int *bc = s->rbc.as<unsigned int>(), *bs = bc + nblk;
    k_starts_count<<<nblk, B, 0, st>>>(s->upal.as<uint8_t>(), s->dfc.as<unsigned long long>(),
                                       s->dft.as<unsigned long long>(), path_of(s->PK.as<unsigned int>(), s->RK.as<unsigned int>()),
                                       s->PM.as<unsigned long long>(), n1, bc, s->cand.as<unsigned long long>(), nullptr,
                                       n0);
    EC_CHECK(scan_incl_u32(s, bc, bs, nblk));
    k_starts_write<<<nblk, B, 0, st>>>(s->upal.as<uint8_t>(), s->dfc.as<unsigned long long>(),
                                       s->dft.as<unsigned long long>(), path_of(s->PK.as<unsigned int>(), s->RK.as<unsigned int>()),
                                       s->PM.as<unsigned long long>(), n1, bs, s->cand.as<unsigned long long>(),
                                       s->skeys.as<unsigned long long>(), s->svals.as<unsigned int>(), n0);
    unsigned int cnt = 0;
    EC_CHECK(d2h(s, &cnt, bs + nblk - 1, 4, st));
    EC_CHECK(host_sync(s, st));
    *n_starts = cnt;
    if (!d_starts) {  // counted only: ec_graph_starts_copy writes them
        s->hold = ec_session::Pending{3, cnt, 0, false};
        return EC_OK;
    }
    return part_starts_copy(s, cnt, d_starts);
}

int part_layout(ec_session *s, const StartRec *d_all, uint64_t nc, uint64_t *n_chars) {
    hipStream_t st = s->stream;
    s->hold.kind = 0;
    const unsigned B = 256;
    const size_t Nn = std::max<size_t>(2 * (size_t)s->n_dense, 1), nn = std::max<size_t>(nc, 1);
    EC_CHECK(s->skeys.ensure(nn * 8));
    EC_CHECK(s->svals.ensure(nn * 4));
    EC_CHECK(s->skeys2.ensure(nn * 8));
    EC_CHECK(s->svals2.ensure(nn * 4));
    EC_CHECK(s->clen.ensure((nn + 1) * 8));
    EC_CHECK(s->coff.ensure((nn + 1) * 8));
    EC_CHECK(s->cwalk.ensure(nn * sizeof(Walk)));
    EC_CHECK(s->cidxOf.ensure(Nn * 4));
    EC_HIP(hipMemsetAsync(s->cidxOf.p, 0xFF, Nn * 4, st));
    EC_HIP(hipMemsetAsync(s->clen.as<unsigned long long>() + nc, 0, 8, st));
    if (nc) {
        k_start_keys<<<grid_for(nc, B), B, 0, st>>>(d_all, (unsigned int)nc, s->skeys.as<unsigned long long>(),
                                                    s->svals.as<unsigned int>());
        EC_CHECK(sort_pairs(s, s->skeys.as<unsigned long long>(), s->skeys2.as<unsigned long long>(),
                            s->svals.as<unsigned int>(), s->svals2.as<unsigned int>(), nc));
        k_layout<<<grid_for(nc, B), B, 0, st>>>(d_all, s->svals2.as<unsigned int>(), (unsigned int)nc,
                                                s->clen.as<unsigned long long>(), s->cidxOf.as<unsigned int>(),
                                                s->cwalk.as<Walk>());
    }
    EC_CHECK(scan_u64(s, s->clen.as<unsigned long long>(), s->coff.as<unsigned long long>(), nc + 1));
    unsigned long long tot = 0;
    EC_CHECK(d2h(s, &tot, s->coff.as<unsigned long long>() + nc, 8, st));
    EC_CHECK(host_sync(s, st));
    s->seg_nc = (unsigned int)nc;
    s->seg_nchars = tot;
    *n_chars = tot;
    return EC_OK;
}

template <typename Ops>
int part_emit(ec_session *s, char *d_chars, void *d_ends, bool check = true) {
    hipStream_t st = s->stream;
    const unsigned B = 256;
    Scalars *dsc = s->scal.as<Scalars>();
    const unsigned int n0 = (unsigned int)s->seg_n0, n1 = (unsigned int)s->seg_n1, nc = s->seg_nc;
    const size_t Nn = std::max<size_t>(2 * (size_t)s->n_dense, 1), nn = std::max<size_t>(nc, 1);
    EC_CHECK(s->cfirst.ensure(nn * 4));
    EC_CHECK(s->clast.ensure(nn * 4));
    EC_CHECK(s->headOf.ensure(Nn * 4));
    EC_CHECK(s->tailOf.ensure(Nn * 4));
    EC_HIP(hipMemsetAsync(s->cfirst.p, 0xFF, nn * 4, st));
    EC_HIP(hipMemsetAsync(s->clast.p, 0xFF, nn * 4, st));
    EC_HIP(hipMemsetAsync(&dsc->skew, 0, 4, st));
    EC_CHECK(s->ewalk.ensure(nn * sizeof(EWalk)));
    if (nc)
        k_ewalk<<<grid_for(nc, B), B, 0, st>>>(s->cwalk.as<Walk>(), s->coff.as<unsigned long long>(), nc,
                                              s->ewalk.as<EWalk>());
    if (n1 > n0 && nc)
        k_emit<Ops><<<grid_for(n1 - n0, B), B, 0, st>>>(
            s->upal.as<uint8_t>(), path_of(s->PK.as<unsigned int>(), s->RK.as<unsigned int>()),
            s->PL.as<unsigned int>(), s->dkey.as<typename Ops::K>(), s->cidxOf.as<unsigned int>(), s->ewalk.as<EWalk>(),
            n1, s->k, d_chars, std::max<uint64_t>(s->seg_nchars, 1),
            s->cfirst.as<unsigned int>(), s->clast.as<unsigned int>(), s->headOf.as<unsigned int>(),
            s->tailOf.as<unsigned int>(), &dsc->skew, n0);
    // contig ends as k-mer codes (the collecting rank holds no global set): 2 nc codes, each
    // written by the rank that emitted the node, zeros elsewhere
    if (nc && d_ends)
        k_ends_codes<Ops><<<grid_for(nc, B), B, 0, st>>>(s->cfirst.as<unsigned int>(), s->clast.as<unsigned int>(), nc,
                                                         s->dkey.as<typename Ops::K>(), s->k,
                                                         reinterpret_cast<typename Ops::K *>(d_ends));
    if (!check) return EC_OK;  // (the caller reads dsc->skew with its own scalars)
    unsigned int bad = 0;
    EC_CHECK(d2h(s, &bad, &dsc->skew, 4, st));
    EC_CHECK(host_sync(s, st));
    if (bad) {
        set_error("contig characters past their bound %llu (inconsistent ranking)", (unsigned long long)s->seg_nchars);
        return EC_ERR_STATE;
    }
    return EC_OK;
}

template <typename Ops>
int part_collect(ec_session *s, const char *d_chars, const void *d_ends_v, uint64_t n_pal, bool packable = false) {
    using K = typename Ops::K;
    using T = typename EndSlotOf<K>::T;
    hipStream_t st = s->stream;
    const unsigned B = 256;
    const unsigned int U = (unsigned int)s->n_dense, nc = s->seg_nc;
    const size_t nn = std::max<size_t>(nc, 1);
    const uint64_t nchars = s->seg_nchars;
    const K *d_ends = static_cast<const K *>(d_ends_v);
    EC_CHECK(s->lk.ensure(nn * 16 * 8));
    EC_CHECK(s->lcnt.ensure(nn * 2 * 4));
    if (nc) {  // GFA links from the contig-end codes (junction.h): a table of 2 nc entries
        uint64_t cap = 1024;
        while (cap < 4ull * nc) cap <<= 1;
        EC_CHECK(s->table.ensure(cap * sizeof(T)));
        T *t = s->table.as<T>();
        if (sizeof(K) == 8) k_end_clear64<<<grid_for(cap, B, 8192), B, 0, st>>>(reinterpret_cast<EndSlot64 *>(t), cap);
        else k_end_clearW<<<grid_for(cap, B, 8192), B, 0, st>>>(reinterpret_cast<EndSlotW *>(t), cap);
        k_end_insert<Ops><<<grid_for(nc, B), B, 0, st>>>(d_ends, nc, s->k, t, cap - 1);
        k_gfa_codes<Ops><<<grid_for(nc, B), B, 0, st>>>(d_ends, nc, s->k, t, cap - 1, s->lk.as<long long>(),
                                                        s->lcnt.as<unsigned int>());
    }
    const unsigned int n2 = 2 * nc;
    s->links_compact = false;
    EC_CHECK(s->h_coff.resize((size_t)nc + 1));
    EC_CHECK(s->h_loff.resize((size_t)n2 + 1));
    s->h_loff[n2] = 0;
    EC_CHECK(d2h(s, s->h_coff.data(), s->coff.p, ((size_t)nc + 1) * 8, st));
    if (nc) {
        EC_CHECK(s->skeys.ensure(((size_t)n2 + 1) * 8));
        EC_CHECK(s->skeys2.ensure(((size_t)n2 + 1) * 8));
        k_lcnt64<<<grid_for(n2 + 1ull, B), B, 0, st>>>(s->lcnt.as<unsigned int>(), n2, s->skeys.as<unsigned long long>());
        EC_CHECK(scan_u64(s, s->skeys.as<unsigned long long>(), s->skeys2.as<unsigned long long>(), (size_t)n2 + 1));
        EC_CHECK(d2h(s, s->h_loff.data(), s->skeys2.p, ((size_t)n2 + 1) * 8, st));
    }
    // (d_chars of the session, 16 B padded: the characters travel as 2-bit codes, as phase_graph's)
    const bool pack = packable && !std::is_same<Ops, OpsX>::value && kn().no_char_pack == 0;
    s->chars_packed = pack;
    s->nchars_host = nchars;
    if (pack) {
        const uint64_t cap16 = (nchars + 15) / 16;
        EC_CHECK(s->dchars.ensure(std::max<uint64_t>(cap16, 1) * 4));
        if (cap16)
            k_pack_chars<<<std::min(grid_for(cap16, B), 8192u), B, 0, st>>>(
                reinterpret_cast<const uint4 *>(d_chars), s->coff.as<unsigned long long>() + nc, cap16,
                s->dchars.as<uint32_t>());
        EC_CHECK(s->h_chars.resize((nchars + 3) / 4));
        if (nchars) EC_CHECK(d2h(s, s->h_chars.data(), s->dchars.p, (nchars + 3) / 4, st));
    } else {
        EC_CHECK(s->h_chars.resize(nchars));
        if (nchars) EC_CHECK(d2h(s, s->h_chars.data(), d_chars, nchars, st));
    }
    EC_CHECK(host_sync(s, st));
    const uint64_t nlinks = s->h_loff[n2];
    EC_CHECK(s->h_links.resize(nlinks));
    if (nlinks) {
        EC_CHECK(s->dcounts.ensure(nlinks * 8));
        k_links_compact<long long><<<grid_for(n2, B), B, 0, st>>>(s->lk.as<long long>(), s->lcnt.as<unsigned int>(),
                                                                 s->skeys2.as<unsigned long long>(), n2,
                                                                 s->dcounts.as<long long>());
        EC_CHECK(d2h(s, s->h_links.data(), s->dcounts.p, nlinks * 8, st));
    }
    EC_CHECK(host_sync(s, st));
    s->stats.n_solid = U;
    s->stats.n_contigs = nc;
    s->stats.n_contig_chars = nchars;
    s->stats.n_links = nlinks;
    s->stats.n_dict = 2ull * U - n_pal;
    s->have = true;
    s->stats_ok = true;
    return EC_OK;
}

// ---- the partitioned finish's transfer to the collecting rank (junction.h, round 6) -----------
// this rank's emission into a zeroed job-sized buffer of its own (never sent), its runs counted
// per chunk and scanned, its contig ends as records; one read-back for the sizes
template <typename Ops>
int part_emit_runs(ec_session *s, uint64_t *nbytes) {
    using K = typename Ops::K;
    hipStream_t st = s->stream;
    const unsigned B = 256;
    Scalars *dsc = s->scal.as<Scalars>();
    const uint64_t nchars = s->seg_nchars;
    const unsigned int nc = s->seg_nc;
    s->runs_ready = false;
    EC_CHECK(s->chars.ensure(nchars + 32));
    EC_HIP(hipMemsetAsync(s->chars.p, 0, nchars + 32, st));
    EC_CHECK(part_emit<Ops>(s, s->chars.as<char>(), nullptr, false));
    const uint64_t nch = (nchars + RUN_CH - 1) / RUN_CH;
    EC_CHECK(s->run_cnt.ensure(4 * (nch + 1) * 8));
    unsigned long long *rc = s->run_cnt.as<unsigned long long>(), *cc = rc + nch + 1, *rb = cc + nch + 1,
                       *cb = rb + nch + 1;
    EC_HIP(hipMemsetAsync(rc, 0, 2 * (nch + 1) * 8, st));
    if (nch) k_runs_count<<<(unsigned)nch, RUN_NT, 0, st>>>(s->chars.as<uint8_t>(), nchars, rc, cc);
    EC_CHECK(scan_u64(s, rc, rb, nch + 1));
    EC_CHECK(scan_u64(s, cc, cb, nch + 1));
    EC_CHECK(s->run_ends.ensure(std::max<size_t>(2ull * nc, 1) * sizeof(EndRec<K>)));
    EC_CHECK(s->jcnt.ensure(16));
    unsigned int *nout = s->jcnt.as<unsigned int>();
    EC_HIP(hipMemsetAsync(nout, 0, 4, st));
    if (nc)
        k_ends_recs<Ops><<<grid_for(nc, B), B, 0, st>>>(s->cfirst.as<unsigned int>(), s->clast.as<unsigned int>(), nc,
                                                        s->dkey.as<K>(), s->k, s->run_ends.as<EndRec<K>>(), nout);
    unsigned long long tot[2] = {0, 0};
    unsigned int ne = 0, bad = 0;
    EC_CHECK(d2h(s, &tot[0], rb + nch, 8, st));
    EC_CHECK(d2h(s, &tot[1], cb + nch, 8, st));
    EC_CHECK(d2h(s, &ne, nout, 4, st));
    EC_CHECK(d2h(s, &bad, &dsc->skew, 4, st));
    EC_CHECK(host_sync(s, st));
    if (bad) {
        set_error("contig characters past their bound %llu (inconsistent ranking)", (unsigned long long)nchars);
        return EC_ERR_STATE;
    }
    s->run_nr = tot[0];
    s->run_nch = tot[1];
    s->run_nends = ne;
    s->runs_ready = true;
    *nbytes = run_rec_bytes(tot[0], tot[1], ne, (int)sizeof(K));
    return EC_OK;
}

// the transfer record into d_out (ec_graph_emit_runs' size), stream-ordered (no sync)
template <typename Ops>
int part_copy_runs(ec_session *s, void *d_out) {
    using K = typename Ops::K;
    hipStream_t st = s->stream;
    const uint64_t nchars = s->seg_nchars, nch = (nchars + RUN_CH - 1) / RUN_CH, nr = s->run_nr;
    unsigned long long *rc = s->run_cnt.as<unsigned long long>(), *rb = rc + 2 * (nch + 1), *cb = rb + nch + 1;
    unsigned long long *hdr = static_cast<unsigned long long *>(d_out);
    unsigned long long *rstart = hdr + 4, *rcoff = rstart + nr;
    uint8_t *rchars = reinterpret_cast<uint8_t *>(rcoff + nr);
    uint8_t *ends = rchars + ((s->run_nch + 7) & ~7ull);
    k_put_u64x4<<<1, 64, 0, st>>>(hdr, nr, s->run_nch, s->run_nends, 0ull);
    if (nch) k_runs_write<<<(unsigned)nch, RUN_NT, 0, st>>>(s->chars.as<uint8_t>(), nchars, rb, cb, rstart, rcoff, rchars);
    if (s->run_nends)
        EC_HIP(hipMemcpyAsync(ends, s->run_ends.p, s->run_nends * sizeof(EndRec<K>), hipMemcpyDeviceToDevice, st));
    return EC_OK;
}

// the collecting rank: every rank's transfer record (concatenated, src_bytes each) into the
// job's characters and end table, then part_collect
template <typename Ops>
int part_collect_runs(ec_session *s, const uint8_t *d_in, int nsrc, const uint64_t *src_bytes, uint64_t n_pal) {
    using K = typename Ops::K;
    hipStream_t st = s->stream;
    const unsigned B = 256;
    const uint64_t nchars = s->seg_nchars;
    const unsigned int nc = s->seg_nc;
    std::vector<unsigned long long> hdr(4 * (size_t)nsrc);
    uint64_t o = 0;
    for (int r = 0; r < nsrc; r++) {
        if (src_bytes[r] < 32 || (o & 7)) {
            set_error("ec_graph_collect_runs: source %d's record is %llu bytes at offset %llu", r,
                      (unsigned long long)src_bytes[r], (unsigned long long)o);
            return EC_ERR_ARG;
        }
        EC_CHECK(d2h(s, &hdr[4 * r], d_in + o, 32, st));
        o += src_bytes[r];
    }
    EC_CHECK(host_sync(s, st));
    EC_CHECK(s->chars.ensure(nchars + 32));
    EC_CHECK(s->run_dends.ensure(std::max<size_t>(2ull * nc, 1) * sizeof(K)));
    EC_HIP(hipMemsetAsync(s->run_dends.p, 0, std::max<size_t>(2ull * nc, 1) * sizeof(K), st));
    EC_CHECK(s->jcnt.ensure(16));
    unsigned int *bad = s->jcnt.as<unsigned int>();
    EC_HIP(hipMemsetAsync(bad, 0, 4, st));
    o = 0;
    for (int r = 0; r < nsrc; r++) {
        const uint64_t nr = hdr[4 * r], nch = hdr[4 * r + 1], ne = hdr[4 * r + 2];
        if (run_rec_bytes(nr, nch, ne, (int)sizeof(K)) != src_bytes[r]) {
            set_error("ec_graph_collect_runs: source %d's record holds %llu bytes, its header %llu", r,
                      (unsigned long long)src_bytes[r], (unsigned long long)run_rec_bytes(nr, nch, ne, (int)sizeof(K)));
            return EC_ERR_ARG;
        }
        const unsigned long long *rstart = reinterpret_cast<const unsigned long long *>(d_in + o) + 4;
        const unsigned long long *rcoff = rstart + nr;
        const uint8_t *rchars = reinterpret_cast<const uint8_t *>(rcoff + nr);
        const EndRec<K> *ends = reinterpret_cast<const EndRec<K> *>(rchars + ((nch + 7) & ~7ull));
        if (nr)
            k_runs_scatter<<<std::min(grid_for(nr, B), 8192u), B, 0, st>>>(rstart, rcoff, nr, nch, rchars,
                                                                         s->chars.as<uint8_t>(), nchars, bad);
        if (ne)
            k_ends_scatter<K><<<grid_for(ne, B), B, 0, st>>>(ends, ne, 2 * nc, s->run_dends.as<K>(), bad);
        o += src_bytes[r];
    }
    unsigned int hb = 0;
    EC_CHECK(d2h(s, &hb, bad, 4, st));
    EC_CHECK(host_sync(s, st));
    if (hb) {
        set_error("ec_graph_collect_runs: a run or an end outside the layout");
        return EC_ERR_ARG;
    }
    return part_collect<Ops>(s, s->chars.as<char>(), s->run_dends.p, n_pal, true);
}

// ---- extended alphabet (extended.h) -----------------------------------------------------------
// c_xa (the symbol table the OpsX kernels read) is one per process: extended-alphabet calls
// of different sessions are serialised (each call ends with its stream synchronised)
std::mutex g_xmu;

int x_upload(ec_session *s) {
    EC_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(c_xa), &s->xa, sizeof(XAlpha), 0, hipMemcpyHostToDevice, s->stream));
    return EC_OK;
}

// the symbol table from the bytes present (bit c of pm): A C G T = 0..3, 'N' the segment split
// (split_n) or an opaque symbol, every other byte an opaque symbol in byte order
int x_alphabet(ec_session *s, const unsigned int *pm, bool split_n, int k) {
    XAlpha &xa = s->xa;
    memset(&xa, 0, sizeof xa);
    const char *acgt = "ACGT";
    for (int c = 0; c < 256; c++) xa.code[c] = 0xFE;
    for (int b = 0; b < 4; b++) xa.code[(int)acgt[b]] = (uint8_t)b, xa.dec[b] = (uint8_t)acgt[b];
    if (split_n) xa.code[(int)'N'] = 0xFF;
    unsigned int nsym = 4;
    for (int c = 0; c < 256; c++)
        if (((pm[c >> 5] >> (c & 31)) & 1u) && xa.code[c] == 0xFE) {
            xa.code[c] = (uint8_t)nsym;
            xa.dec[nsym++] = (uint8_t)c;
        }
    xa.nsym = nsym;
    xa.sb = nsym <= 16 ? 4 : nsym <= 32 ? 5 : 8;
    if (xa.sb * (unsigned)k > 126) {
        set_error("the input holds %u symbols besides A/C/G/T%s (%u bits each): k = %d needs %u-bit keys, more than "
                  "126 (k <= %u for this alphabet)", nsym - 4, split_n ? "/N" : "", xa.sb, k, xa.sb * k, 126 / xa.sb);
        return EC_ERR_ALPHABET;
    }
    EC_CHECK(x_upload(s));
    s->xalpha = true;
    return EC_OK;
}

// all_contigs on a caller's dict holding bytes other than A/C/G/T (ec_assemble_from_kmers)
int assemble_kmers_extended(ec_session *s, const char *kmers, uint64_t n, int k) {
    std::lock_guard<std::mutex> lock(g_xmu);
    unsigned int pm[8] = {};
    for (uint64_t i = 0; i < n * (uint64_t)k; i++) {
        const unsigned char c = (unsigned char)kmers[i];
        pm[c >> 5] |= 1u << (c & 31);
    }
    EC_CHECK(x_alphabet(s, pm, false, k));
    hipStream_t st = s->stream;
    k_x_kmers_to_agg<<<grid_for(n, 256), 256, 0, st>>>(s->dchars.as<char>(), s->dcounts.as<unsigned int>(), n, k,
                                                       s->recs2.as<AggW>());
    unsigned int U = 0;
    SolidIndexW sidx{};
    EC_CHECK(phase_merge_w(s, s->recs2.as<AggW>(), n, LLONG_MIN, U, sidx));
    return phase_graph<OpsX>(s, k, U, sidx);
}

// reads with bytes other than A/C/G/T/N: symbol table from the bytes present, count into the
// wide HBM table (128-bit keys of sb-bit symbols), then the graph phase over OpsX
int assemble_extended(ec_session *s, const uint8_t *d_reads, const uint64_t *d_off, uint64_t nreads, int k,
                      long long limit) {
    std::lock_guard<std::mutex> lock(g_xmu);
    hipStream_t st = s->stream;
    const unsigned B = 256;
    Scalars *dsc = s->scal.as<Scalars>();
    Scalars hsc;
    EC_CHECK(s->tmp.ensure(64));
    unsigned int *present = s->tmp.as<unsigned int>();
    EC_HIP(hipMemsetAsync(present, 0, 32, st));
    if (nreads) k_x_alphabet<<<grid_for(nreads, B, 4096), B, 0, st>>>(d_reads, d_off, nreads, present);
    unsigned int pm[8];
    EC_CHECK(d2h(s, pm, present, 32, st));
    EC_CHECK(host_sync(s, st));
    EC_CHECK(x_alphabet(s, pm, true, k));
    s->stats.count_variant = 0;
    s->stats.n_buckets = 0;
    s->stats.record_bytes = 0;
    s->stats.n_records = 0;
    s->stats.n_reads = nreads;
    // prescan (positions, HyperLogLog of the canonical keys) + count (phase_count_w's table)
    mark(s, 2 * EC_STAGE_PRESCAN);
    EC_CHECK(s->hll.ensure(HLL_M * 4));
    EC_HIP(hipMemsetAsync(s->hll.p, 0, HLL_M * 4, st));
    EC_HIP(hipMemsetAsync(&dsc->npos, 0, 8, st));
    EC_HIP(hipMemsetAsync(&dsc->est, 0, 8, st));
    if (nreads) {
        k_x_prescan<<<grid_for(nreads, B, 4096), B, 0, st>>>(d_reads, d_off, nreads, k, s->hll.as<unsigned int>(),
                                                            &dsc->npos);
        k_hll_final<<<1, 1024, 0, st>>>(s->hll.as<unsigned int>(), HLL_BITS, &dsc->est);
    }
    mark(s, 2 * EC_STAGE_PRESCAN + 1);
    EC_CHECK(d2h(s, &hsc, dsc, sizeof(Scalars), st));
    EC_CHECK(host_sync(s, st));
    const uint64_t P = nreads ? hsc.npos : 0;
    s->stats.n_positions = P;
    const double est = nreads ? hsc.est : 0.0;
    s->stats.n_distinct_est = (uint64_t)llround(est);
    uint64_t cap = 1024;
    const double want = std::min((double)P, 1.05 * est) * 1.6 + 1024;
    while ((double)cap < want) cap <<= 1;
    for (int attempt = 0;; attempt++) {
        EC_CHECK(s->table.ensure(cap * sizeof(SlotW)));
        mark(s, 2 * EC_STAGE_COUNT);
        k_table_clear_w<<<grid_for(cap, B, 8192), B, 0, st>>>(s->table.as<SlotW>(), cap);
        EC_HIP(hipMemsetAsync(&dsc->overflow, 0, 4, st));
        if (nreads) {
            kmark(s, 3, 0);
            k_x_count<<<grid_for(nreads, B), B, 0, st>>>(d_reads, d_off, nreads, k, s->table.as<SlotW>(), cap - 1,
                                                        &dsc->overflow);
            kmark(s, 3, 1);
        }
        mark(s, 2 * EC_STAGE_COUNT + 1);
        EC_CHECK(d2h(s, &hsc.overflow, &dsc->overflow, 4, st));
        EC_CHECK(host_sync(s, st));
        if (!hsc.overflow) break;
        if (attempt >= 4) {
            set_error("hash table overflow at capacity %llu", (unsigned long long)cap);
            return EC_ERR_CAPACITY;
        }
        cap <<= 2;
        s->stats.table_retries++;
    }
    unsigned int U = 0;
    SolidIndexW sidx{};
    EC_CHECK(finish_wide(s, cap, limit, U, sidx));
    return phase_graph<OpsX>(s, k, U, sidx);
}

int assemble(ec_session *s, const uint8_t *d_reads, const uint64_t *d_off, uint64_t nreads, int k, int limit,
             unsigned flags) {
    EC_CHECK(begin_call(s, k, flags));
    unsigned int U = 0;
    if (k > 32) {
        SolidIndexW sidx{};
        EC_CHECK(pipe_all(s));
        const int rc = phase_count_w(s, d_reads, d_off, nreads, 0, k, (long long)limit, U, sidx);
        if (rc == EC_ERR_ALPHABET) return assemble_extended(s, d_reads, d_off, nreads, k, (long long)limit);
        EC_CHECK(rc);
        return phase_graph<OpsW>(s, k, U, sidx);
    }
    SolidIndex sidx{};
    const int rc = phase_count(s, d_reads, d_off, nreads, 0, k, (long long)limit, flags, U, sidx);
    if (rc == EC_ERR_ALPHABET) {  // bytes other than A/C/G/T/N: opaque symbols (extended.h)
        EC_CHECK(pipe_all(s));
        return assemble_extended(s, d_reads, d_off, nreads, k, (long long)limit);
    }
    EC_CHECK(rc);
    return phase_graph<Ops64>(s, k, U, sidx);
}

// ---- host input -------------------------------------------------------------------------------
using Pipe = ec_session::Pipe;
// Chunk plan over nbases bases (chunk boundaries at multiples of 64 bases, ~32 MiB of copied
// bytes a chunk) and the reads each chunk completes (offsets: host array, or NULL = one length L)
int pipe_plan(ec_session *s, Pipe &pp, uint64_t nbases, uint64_t bytes_per_base4, const uint64_t *offsets,
              uint64_t nreads, uint64_t L, hipEvent_t after = nullptr) {
    const uint64_t copy_bytes = bytes_per_base4 ? (nbases + 3) / 4 : nbases;
    int nc = (int)std::min<uint64_t>(64, std::max<uint64_t>(1, copy_bytes >> 25));
    if (kn().host_chunks) nc = std::max(1, std::min(64, kn().host_chunks));
    pp.nchunks = nc;
    pp.done = 0;
    pp.blo.assign(nc, 0), pp.bhi.assign(nc, 0), pp.ravail.assign(nc, 0), pp.elo.assign(nc, 0), pp.ehi.assign(nc, 0);
    for (int c = 0; c < nc; c++) {
        pp.blo[c] = c ? pp.bhi[c - 1] : 0;
        pp.bhi[c] = c + 1 == nc ? nbases : std::max<uint64_t>(pp.blo[c], (nbases * (uint64_t)(c + 1) / nc) & ~63ull);
        uint64_t r;  // reads with offsets[r + 1] <= bhi
        if (c + 1 == nc) r = nreads;
        else if (!offsets) r = L ? std::min<uint64_t>(nreads, pp.bhi[c] / L) : nreads;
        else r = (uint64_t)(std::upper_bound(offsets + 1, offsets + nreads + 1, pp.bhi[c]) - (offsets + 1));
        pp.ravail[c] = r;
    }
    if ((int)pp.ev.size() < nc) {
        const size_t have = pp.ev.size();
        pp.ev.resize(nc, nullptr);
        for (size_t i = have; i < (size_t)nc; i++) EC_HIP(hipEventCreateWithFlags(&pp.ev[i], hipEventDisableTiming));
    }
    if (!s->cstream) EC_HIP(hipStreamCreateWithFlags(&s->cstream, hipStreamNonBlocking));
    if (!s->cstream2) EC_HIP(hipStreamCreateWithFlags(&s->cstream2, hipStreamNonBlocking));
    // the copies overwrite buffers a previous call's kernels may still read: after = the event
    // of their last reader (a staged slot), else everything queued on the session stream
    if (!after) {
        EC_HIP(hipEventRecord(pp.ev[0], s->stream));
        after = pp.ev[0];
    }
    EC_HIP(hipStreamWaitEvent(s->cstream, after, 0));
    EC_HIP(hipStreamWaitEvent(s->cstream2, after, 0));
    return EC_OK;
}

// the copy stream of chunk c (EULERHIP_COPY_STREAMS=1: cstream only)
inline hipStream_t copy_stream(ec_session *s, int c) { return (c & 1) && kn().copy_streams == 2 ? s->cstream2 : s->cstream; }

// copy the offsets entries reads [r0, r1] need (chunk by chunk: [ravail[c-1] + 1, ravail[c] + 1))
int pipe_copy_offsets(ec_session *s, const Pipe &pp, int c, const uint64_t *offsets, uint64_t *d_off) {
    const uint64_t o0 = c ? pp.ravail[c - 1] + 1 : 0, o1 = pp.ravail[c] + 1;
    if (o1 > o0)
        EC_HIP(hipMemcpyAsync(d_off + o0, offsets + o0, (o1 - o0) * 8, hipMemcpyHostToDevice, copy_stream(s, c)));
    return EC_OK;
}

int check_offsets(const uint64_t *offsets, uint64_t nreads, uint64_t nbytes) {
    if (offsets[nreads] > nbytes) {
        set_error("offsets[nreads]=%llu > nbytes=%llu", (unsigned long long)offsets[nreads], (unsigned long long)nbytes);
        return EC_ERR_ARG;
    }
    for (uint64_t i = 0; i < nreads; i++)
        if (offsets[i] > offsets[i + 1]) {
            set_error("offsets not monotone at %llu", (unsigned long long)i);
            return EC_ERR_ARG;
        }
    return EC_OK;
}

// run assemble() on the pipelined input; the pipeline is drained (every chunk consumed) on any
// return so no chunk copy is left pending against the next call's buffers
int assemble_piped(ec_session *s, const uint64_t *d_off, uint64_t nreads, int k, int limit, unsigned flags) {
    s->pipe.active = true;
    s->pipe.ascii = s->h_reads.as<uint8_t>();  // (staged batches: h_reads may have grown since)
    int rc = EC_OK;
    // copies already complete (a staged batch, copied while the previous one assembled): the
    // count runs once over the whole batch -- per-chunk partition launches fill the chip only
    // a seventh at a time (7 x 0.34 ms against 0.98 ms for one launch at the headline)
    if (s->pipe.nchunks > 1 && s->pipe.done < s->pipe.nchunks &&
        hipEventQuery(s->pipe.ev[s->pipe.nchunks - 1]) == hipSuccess)
        rc = pipe_all(s);
    if (rc == EC_OK) rc = assemble(s, s->h_reads.as<uint8_t>(), d_off, nreads, k, limit, flags);
    if (s->pipe.done < s->pipe.nchunks) {
        pipe_all(s);
        (void)host_sync(s, s->stream);
    }
    s->pipe.active = false;
    return rc;
}

int check_packed(const uint8_t *codes, uint64_t nbases, const uint64_t *offsets, uint64_t nreads, uint32_t read_len,
                 const uint64_t *exc_pos, const uint8_t *exc_byte, uint64_t n_exc) {
    if ((nbases && !codes) || (n_exc && (!exc_pos || !exc_byte))) {
        set_error("null argument");
        return EC_ERR_ARG;
    }
    if (offsets) {
        EC_CHECK(check_offsets(offsets, nreads, nbases));
    } else if ((uint64_t)read_len * nreads != nbases) {
        set_error("%llu reads of %u bases != %llu bases", (unsigned long long)nreads, read_len,
                  (unsigned long long)nbases);
        return EC_ERR_ARG;
    }
    for (uint64_t i = 0; i < n_exc; i++)
        if (exc_pos[i] >= nbases || (i && exc_pos[i] <= exc_pos[i - 1])) {
            set_error("exception %llu: position %llu not ascending inside [0, %llu)", (unsigned long long)i,
                      (unsigned long long)exc_pos[i], (unsigned long long)nbases);
            return EC_ERR_ARG;
        }
    return EC_OK;
}

// a packed batch's copies into (codes_b, exc_b, off_b) on cstream, chunk events in pp (the
// plan of assemble_piped); after = the event the copies wait for (nullptr: the session stream)
int stage_packed(ec_session *s, Pipe &pp, DevBuf &codes_b, DevBuf &exc_b, DevBuf &off_b, hipEvent_t after,
                 const uint8_t *codes, uint64_t nbases, const uint64_t *offsets, uint64_t nreads, uint32_t read_len,
                 const uint64_t *exc_pos, const uint8_t *exc_byte, uint64_t n_exc) {
    const uint64_t ncodes = (nbases + 3) / 4;
    EC_CHECK(off_b.ensure((nreads + 1) * 8));
    EC_CHECK(codes_b.ensure(((ncodes + 3) & ~3ull) + 16));
    EC_CHECK(exc_b.ensure(n_exc * 9 + 16));
    EC_CHECK(pipe_plan(s, pp, nbases, 1, offsets, nreads, read_len, after));
    pp.packed = true;
    pp.first_len = nreads ? (offsets ? offsets[1] - offsets[0] : read_len) : 0;
    pp.codes = codes_b.as<uint32_t>();
    pp.exc_pos = exc_b.as<uint64_t>();
    pp.exc_byte = exc_b.as<uint8_t>() + n_exc * 8;
    if (n_exc) {
        EC_HIP(hipMemcpyAsync(exc_b.p, exc_pos, n_exc * 8, hipMemcpyHostToDevice, s->cstream));
        EC_HIP(hipMemcpyAsync(exc_b.as<uint8_t>() + n_exc * 8, exc_byte, n_exc, hipMemcpyHostToDevice, s->cstream));
    }
    if (!offsets)  // one read length: the offsets are made on the device (ordered before chunk 0's event)
        k_iota_off<<<grid_for(nreads + 1, 256, 16384), 256, 0, s->cstream>>>(off_b.as<uint64_t>(), nreads + 1, read_len);
    for (int c = 0; c < pp.nchunks; c++) {
        // code bytes of bases [blo, bhi) (blo a multiple of 64: whole 32-bit words)
        const uint64_t c0 = pp.blo[c] / 4, c1 = c + 1 == pp.nchunks ? ncodes : pp.bhi[c] / 4;
        if (c1 > c0)
            EC_HIP(hipMemcpyAsync(codes_b.as<uint8_t>() + c0, codes + c0, c1 - c0, hipMemcpyHostToDevice,
                                  copy_stream(s, c)));
        if (offsets) EC_CHECK(pipe_copy_offsets(s, pp, c, offsets, off_b.as<uint64_t>()));
        pp.elo[c] = (uint64_t)(std::lower_bound(exc_pos, exc_pos + n_exc, pp.blo[c]) - exc_pos);
        pp.ehi[c] = (uint64_t)(std::lower_bound(exc_pos, exc_pos + n_exc, pp.bhi[c]) - exc_pos);
        EC_HIP(hipEventRecord(pp.ev[c], copy_stream(s, c)));
    }
    return EC_OK;
}

}  // namespace

// 2-bit codes (4 a byte, first character in the low bits) -> n ASCII characters; threads past
// ~4 MB of characters (ecoli10m_err: 38 MB)
static void unpack_codes(const uint8_t *codes, uint64_t n, char *out) {
    static const struct Lut {
        uint32_t v[256];
        Lut() {
            const char acgt[4] = {'A', 'C', 'G', 'T'};
            for (int b = 0; b < 256; b++) {
                uint32_t w = 0;
                for (int j = 0; j < 4; j++) w |= (uint32_t)(uint8_t)acgt[(b >> (2 * j)) & 3] << (8 * j);
                v[b] = w;
            }
        }
    } lut;
    auto run = [&](uint64_t b0, uint64_t b1) {  // whole bytes [b0, b1) -> characters 4 b0 ..
        for (uint64_t i = b0; i < b1; i++) memcpy(out + 4 * i, &lut.v[codes[i]], 4);
    };
    const uint64_t full = n / 4;
    const unsigned nt = full >= (1ull << 20) ? std::max(1u, std::min(16u, std::thread::hardware_concurrency())) : 1u;
    if (nt > 1) {
        std::vector<std::thread> th;
        for (unsigned t = 0; t < nt; t++) th.emplace_back(run, full * t / nt, full * (t + 1) / nt);
        for (auto &x : th) x.join();
    } else {
        run(0, full);
    }
    for (uint64_t c = 4 * full; c < n; c++) out[c] = "ACGT"[(codes[full] >> (2 * (c & 3))) & 3];
}

// every device buffer of a session (destroy, trim)
template <typename Fn>
static void for_each_buf(ec_session *s, Fn fn) {
    DevBuf *all[] = {&s->h_reads, &s->h_offsets, &s->hll, &s->scal, &s->table, &s->dkey, &s->dcnt, &s->dfc, &s->dft,
                     &s->upal, &s->outdeg, &s->cand, &s->succ, &s->pred, &s->st0, &s->st1, &s->startOf, &s->skeys,
                     &s->svals, &s->skeys2, &s->svals2, &s->cidxOf, &s->clen, &s->coff, &s->chars, &s->cfirst,
                     &s->clast, &s->headOf, &s->tailOf, &s->lk, &s->lcnt, &s->tmp, &s->dchars, &s->dcounts,
                     &s->rid, &s->rlist, &s->nextR, &s->PK, &s->RK, &s->PL, &s->PM,
                     &s->ocnt, &s->hist, &s->ftot, &s->cnt, &s->offs, &s->bstart, &s->tot, &s->recs, &s->recs2, &s->sub, &s->bnp, &s->rbc,
                     &s->mbid, &s->mbid2, &s->midx, &s->midx2, &s->gcur, &s->cwalk, &s->ewalk, &s->lc8, &s->x_par, &s->x_irr,
                     &s->x_in, &s->x_succ, &s->x_done, &s->x_lk, &s->x_lv, &s->x_lk2, &s->x_lv2, &s->x_len,
                     &s->x_m, &s->x_cid, &s->x_head, &s->x_tail, &s->rt_tcnt, &s->rt_tbase, &s->rt_srec,
                     &s->rt_snrec, &s->rt_sidx, &s->rt_pks, &s->rt_rks, &s->rt_hasp, &s->rt_lr, &s->wbv, &s->bmark, &s->rt_tb,
                     &s->jrec, &s->joid, &s->jout, &s->jseg, &s->jcnt, &s->xrec,
                     &s->skm_rec, &s->skm_ev, &s->skm_end, &s->wcodes_tab,
                     &s->run_cnt, &s->run_ends, &s->run_dends, &s->rt_lb,
                     &s->jl_kof, &s->jl_rs, &s->jl_re, &s->jl_cnt, &s->jl_off, &s->jl_flag, &s->rpack};
    for (auto *b : all) fn(*b);
}

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
    EC_HIP(hipSetDevice(s->device));
    if (hip_stream == EC_OWN_STREAM) {
        if (!s->own_stream) {
            EC_HIP(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
            s->own_stream = true;
        }
        return EC_OK;
    }
    if (s->own_stream && s->stream) {
        (void)host_sync(s, s->stream);
        hipStreamDestroy(s->stream);
    }
    s->own_stream = false;
    s->stream = (hipStream_t)hip_stream;  // NULL: the null stream
    return EC_OK;
}

uint64_t ec_session_bytes(ec_session *s) {
    uint64_t n = 0;
    if (s) for_each_buf(s, [&](DevBuf &b) { n += b.cap; });
    return n;
}

int ec_session_trim(ec_session *s, uint64_t min_bytes) {
    if (!s) return EC_ERR_ARG;
    EC_HIP(hipSetDevice(s->device));
    if (s->stream) EC_HIP(hipStreamSynchronize(s->stream));
    if (s->ostream) EC_HIP(hipStreamSynchronize(s->ostream));
    if (s->cstream) EC_HIP(hipStreamSynchronize(s->cstream));
    if (s->cstream2) EC_HIP(hipStreamSynchronize(s->cstream2));
    for_each_buf(s, [&](DevBuf &b) {
        if (b.cap >= min_bytes && &b != &s->scal) b.release();
    });
    // no device state survives: the next call starts from its inputs (results already copied to
    // host memory stay fetchable)
    s->n_dense = 0;
    s->own_valid = false;
    s->bmark_ok = false;
    s->seg_marks = 0;
    s->skspec.valid = false;
    s->graph_loaded = false;
    s->placed = false;
    s->pipe.active = false;
    return EC_OK;
}

int ec_mem_stats(uint64_t *held, uint64_t *peak, int reset) {
    if (held) *held = g_hbm_held.load();
    if (peak) *peak = g_hbm_peak.load();
    if (reset) g_hbm_peak.store(g_hbm_held.load());
    return EC_OK;
}

int ec_session_destroy(ec_session *s) {
    if (!s) return EC_OK;
    hipSetDevice(s->device);
    // every stream that may still copy into / out of the session's buffers (the speculative
    // contig copy on ostream, staged batches on cstream) drains before anything is released
    if (s->stream) hipStreamSynchronize(s->stream);
    if (s->ostream) hipStreamSynchronize(s->ostream);
    if (s->cstream) hipStreamSynchronize(s->cstream);
    if (s->cstream2) hipStreamSynchronize(s->cstream2);
    for_each_buf(s, [](DevBuf &b) { b.release(); });
    s->h_chars.release();
    s->hmeta.release();
    s->bounce.release();
    s->pend.clear();
    s->h_coff.release();
    s->h_loff.release();
    s->h_links.release();
    s->h_lc8.release();
    s->h_links32.release();
    if (s->events) {
        for (auto &e : s->ev) hipEventDestroy(e);
        for (auto &e : s->kev) hipEventDestroy(e);
    }
    s->p_codes.release();
    s->p_exc.release();
    if (s->rd_ev) hipEventDestroy(s->rd_ev);
    if (s->ostream) {
        hipStreamSynchronize(s->ostream);
        hipStreamDestroy(s->ostream);
    }
    for (auto &e : s->oev)
        if (e) hipEventDestroy(e);
    for (auto &e : s->pipe.ev) hipEventDestroy(e);
    for (auto &sl : s->stg) {
        for (auto &e : sl.pipe.ev) hipEventDestroy(e);
        if (sl.free_ev) hipEventDestroy(sl.free_ev);
        sl.codes.release();
        sl.exc.release();
        sl.off.release();
    }
    if (s->cstream) {
        hipStreamSynchronize(s->cstream);
        hipStreamDestroy(s->cstream);
    }
    if (s->cstream2) {
        hipStreamSynchronize(s->cstream2);
        hipStreamDestroy(s->cstream2);
    }
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
    refresh_knobs();
    if (!s || !offsets || (nbytes && !reads)) {
        set_error("null argument");
        return EC_ERR_ARG;
    }
    EC_CHECK(check_offsets(offsets, nreads, nbytes));
    EC_HIP(hipSetDevice(s->device));
    EC_CHECK(s->h_reads.ensure(nbytes + 16));
    EC_CHECK(s->h_offsets.ensure((nreads + 1) * 8));
    // chunked copies (reads and offsets) on the copy stream, the partition of the reads that
    // have arrived overlapping the copies of the rest (s->pipe)
    EC_CHECK(pipe_plan(s, s->pipe, nbytes, 0, offsets, nreads, 0));
    auto &pp = s->pipe;
    pp.packed = false;
    pp.first_len = nreads ? offsets[1] - offsets[0] : 0;
    pp.ascii = s->h_reads.as<uint8_t>();
    for (int c = 0; c < pp.nchunks; c++) {
        if (pp.bhi[c] > pp.blo[c])
            EC_HIP(hipMemcpyAsync(s->h_reads.as<uint8_t>() + pp.blo[c], reads + pp.blo[c], pp.bhi[c] - pp.blo[c],
                                  hipMemcpyHostToDevice, copy_stream(s, c)));
        EC_CHECK(pipe_copy_offsets(s, pp, c, offsets, s->h_offsets.as<uint64_t>()));
        EC_HIP(hipEventRecord(pp.ev[c], copy_stream(s, c)));
    }
    return assemble_piped(s, s->h_offsets.as<uint64_t>(), nreads, k, limit, flags);
}

int ec_assemble_packed_host(ec_session *s, const uint8_t *codes, uint64_t nbases, const uint64_t *offsets,
                            uint64_t nreads, uint32_t read_len, const uint64_t *exc_pos, const uint8_t *exc_byte,
                            uint64_t n_exc, int k, int limit, unsigned flags) {
    refresh_knobs();
    if (!s) {
        set_error("null session");
        return EC_ERR_ARG;
    }
    if (s->stg_n) {
        set_error("staged batches pending (ec_assemble_staged first)");
        return EC_ERR_STATE;
    }
    EC_CHECK(check_packed(codes, nbases, offsets, nreads, read_len, exc_pos, exc_byte, n_exc));
    EC_HIP(hipSetDevice(s->device));
    EC_CHECK(s->h_reads.ensure(nbases + 16));
    EC_CHECK(stage_packed(s, s->pipe, s->p_codes, s->p_exc, s->h_offsets, nullptr, codes, nbases, offsets, nreads,
                          read_len, exc_pos, exc_byte, n_exc));
    return assemble_piped(s, s->h_offsets.as<uint64_t>(), nreads, k, limit, flags);
}

int ec_stage_packed_host(ec_session *s, const uint8_t *codes, uint64_t nbases, const uint64_t *offsets,
                         uint64_t nreads, uint32_t read_len, const uint64_t *exc_pos, const uint8_t *exc_byte,
                         uint64_t n_exc) {
    refresh_knobs();
    if (!s) {
        set_error("null session");
        return EC_ERR_ARG;
    }
    if (s->stg_n >= 2) {
        set_error("two batches already staged (ec_assemble_staged first)");
        return EC_ERR_STATE;
    }
    EC_CHECK(check_packed(codes, nbases, offsets, nreads, read_len, exc_pos, exc_byte, n_exc));
    EC_HIP(hipSetDevice(s->device));
    auto &sl = s->stg[(s->stg_head + s->stg_n) & 1];
    if (!sl.free_ev) {  // first use: free once the session stream's current work is done
        EC_HIP(hipEventCreateWithFlags(&sl.free_ev, hipEventDisableTiming));
        EC_HIP(hipEventRecord(sl.free_ev, s->stream));
    }
    EC_CHECK(stage_packed(s, sl.pipe, sl.codes, sl.exc, sl.off, sl.free_ev, codes, nbases, offsets, nreads, read_len,
                          exc_pos, exc_byte, n_exc));
    sl.nreads = nreads;
    sl.nbases = nbases;
    s->stg_n++;
    return EC_OK;
}

int ec_assemble_staged(ec_session *s, int k, int limit, unsigned flags) {
    refresh_knobs();
    if (!s) {
        set_error("null session");
        return EC_ERR_ARG;
    }
    if (!s->stg_n) {
        set_error("no staged batch (ec_stage_packed_host)");
        return EC_ERR_STATE;
    }
    EC_HIP(hipSetDevice(s->device));
    auto &sl = s->stg[s->stg_head];
    int rc = s->h_reads.ensure(sl.nbases + 16);
    if (rc == EC_OK) {
        std::swap(s->pipe, sl.pipe);
        rc = assemble_piped(s, sl.off.as<uint64_t>(), sl.nreads, k, limit, flags);
        std::swap(s->pipe, sl.pipe);
    }
    // the slot is free for the next staged batch once this call's kernels are done with it
    // (drained on every return, so also after a failure)
    if (sl.pipe.done < sl.pipe.nchunks) {  // (a failure before any chunk was consumed)
        for (int c = 0; c < sl.pipe.nchunks; c++) hipStreamWaitEvent(s->stream, sl.pipe.ev[c], 0);
    }
    hipEventRecord(sl.free_ev, s->stream);
    s->stg_head ^= 1;
    s->stg_n--;
    return rc;
}

int ec_get_stats(ec_session *s, ec_stats *out) {
    if (!s || !out) return EC_ERR_ARG;
    if (!s->stats_ok) {
        set_error("no successful call in this session");
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
    if (chars && s->nchars_host) {
        if (s->chars_packed) unpack_codes(reinterpret_cast<const uint8_t *>(s->h_chars.data()), s->nchars_host, chars);
        else memcpy(chars, s->h_chars.data(), s->nchars_host);
    }
    if (offsets) memcpy(offsets, s->h_coff.data(), s->h_coff.size() * 8);
    return EC_OK;
}

int ec_copy_links(ec_session *s, uint64_t *link_offsets, int64_t *links) {
    if (!s) return EC_ERR_ARG;
    if (!s->have) {
        set_error("no successful assembly in this session");
        return EC_ERR_STATE;
    }
    if (s->links_compact) {  // (phase_graph's transfer form: widened here)
        if (link_offsets) {
            uint64_t o = 0;
            const size_t n2 = s->h_lc8.size();
            for (size_t i = 0; i < n2; i++) {
                link_offsets[i] = o;
                o += s->h_lc8[i];
            }
            link_offsets[n2] = o;
        }
        if (links)
            for (size_t i = 0; i < s->h_links32.size(); i++) links[i] = (int64_t)s->h_links32[i];
        return EC_OK;
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
    EC_CHECK(d2h(s, &nd, &dsc->ndict, 4, st));
    EC_CHECK(host_sync(s, st));
    EC_CHECK(sort_pairs(s, s->skeys.as<unsigned long long>(), s->skeys2.as<unsigned long long>(),
                        s->svals.as<unsigned int>(), s->svals2.as<unsigned int>(), nd));
    EC_CHECK(s->dchars.ensure((size_t)nd * s->k));
    EC_CHECK(s->dcounts.ensure((size_t)nd * 4));
    std::unique_lock<std::mutex> xlock(g_xmu, std::defer_lock);
    if (s->xalpha) {  // (c_xa may hold another session's alphabet by now)
        xlock.lock();
        EC_CHECK(x_upload(s));
        k_dict_render<OpsX><<<grid_for(nd, B), B, 0, st>>>(s->svals2.as<unsigned int>(), nd, s->dkey.as<K128>(),
                                                          s->dcnt.as<unsigned int>(), s->k, s->dchars.as<char>(),
                                                          s->dcounts.as<unsigned int>());
    } else if (s->k > 32)
        k_dict_render<OpsW><<<grid_for(nd, B), B, 0, st>>>(s->svals2.as<unsigned int>(), nd, s->dkey.as<K128>(),
                                                          s->dcnt.as<unsigned int>(), s->k, s->dchars.as<char>(),
                                                          s->dcounts.as<unsigned int>());
    else
        k_dict_render<Ops64><<<grid_for(nd, B), B, 0, st>>>(s->svals2.as<unsigned int>(), nd,
                                                           s->dkey.as<unsigned long long>(), s->dcnt.as<unsigned int>(),
                                                           s->k, s->dchars.as<char>(), s->dcounts.as<unsigned int>());
    if (kmers) EC_CHECK(d2h(s, kmers, s->dchars.p, (size_t)nd * s->k, st));
    if (counts) EC_CHECK(d2h(s, counts, s->dcounts.p, (size_t)nd * 4, st));
    EC_CHECK(host_sync(s, st));
    return EC_OK;
}


// ---- sharded (multi-GPU) building blocks ---------------------------------------------------
int ec_count_shard(ec_session *s, const uint8_t *d_reads, const uint64_t *d_offsets, uint64_t nreads,
                   uint64_t read_base, int k, unsigned flags) {
    if (!s || !d_offsets) {
        set_error("null session/offsets");
        return EC_ERR_ARG;
    }
    EC_CHECK(begin_call(s, k, flags));
    if (read_base + nreads > (1ull << 32)) {
        set_error("global read ids reach %llu >= 2^32", (unsigned long long)(read_base + nreads));
        return EC_ERR_CAPACITY;
    }
    unsigned int U = 0;
    s->no_index = true;
    int rc = EC_OK;
    // the shard is counted with shard-relative read ids (so every rank qualifies for the
    // super-k-mer path's 32-bit positions, count_sk2.h); first events are events
    // (read << 32) | window, so the export adds read_base << 32 to every real event
    if (k > 32) {
        SolidIndexW sidx{};
        rc = phase_count_w(s, d_reads, d_offsets, nreads, 0, k, LLONG_MIN, U, sidx);
    } else {
        SolidIndex sidx{};
        rc = phase_count(s, d_reads, d_offsets, nreads, 0, k, LLONG_MIN, flags, U, sidx);
    }
    s->no_index = false;
    EC_CHECK(rc);
    s->shard_base = read_base;
    s->n_dense = U;
    collect_timing(s);
    s->stats_ok = true;
    return EC_OK;
}

int ec_session_set_owner_rule(ec_session *s, int rule) {
    if (!s || rule < 0 || rule > 1) {
        set_error("bad owner rule %d", rule);
        return EC_ERR_ARG;
    }
    if (rule != s->owner_rule) s->own_valid = false;
    s->owner_rule = rule;
    return EC_OK;
}

int ec_export_by_owner(ec_session *s, int nowners, void *d_out, uint64_t *owner_counts) {
    return ec_export_by_owner_ex(s, nowners, d_out, owner_counts, 0, nullptr);
}

int ec_export_by_owner_ex(ec_session *s, int nowners, void *d_out, uint64_t *owner_counts, int compact,
                          int *lf_bits) {
    refresh_knobs();
    if (!s || nowners < 1 || nowners > MAX_OWNERS || !owner_counts) {
        set_error("bad ec_export_by_owner arguments (nowners=%d)", nowners);
        return EC_ERR_ARG;
    }
    EC_HIP(hipSetDevice(s->device));
    hipStream_t st = s->stream;
    const unsigned B = 256;
    const unsigned int n = s->n_dense;
    const unsigned int nblk = (unsigned int)std::max<uint64_t>((n + OWN_CHUNK - 1) / OWN_CHUNK, 1);
    const size_t nbh = (size_t)nowners * nblk;
    EC_CHECK(s->ocnt.ensure(2 * nbh * 4));
    unsigned int *bh = s->ocnt.as<unsigned int>(), *bhi = bh + nbh;
    const bool wide = s->k > 32;
    OwnerFn own = owner_fn(s->k);
    if (s->owner_rule == 1) own.sk = 0, own.wk = 0;  // key-hash owners (a skewed minimizer distribution)
    EC_CHECK(s->mbid.ensure(std::max<uint64_t>(n, 1) * 4));  // owner of each record (free until a merge)
    EC_CHECK(s->ocnt.ensure(2 * nbh * 4 + 16));
    bh = s->ocnt.as<unsigned int>(), bhi = bh + nbh;
    unsigned int *evmax = bhi + nbh;  // largest shard-relative read id / position of the events
    unsigned int *oid = s->mbid.as<unsigned int>();
    const bool reuse = s->own_valid && s->own_rule == s->owner_rule && s->own_nowners == nowners && s->own_n == n &&
                       s->own_nblk == nblk;
    if (!reuse) {
        s->own_hi.assign(nbh + 2, 0u);
        if (n) {
            EC_HIP(hipMemsetAsync(evmax, 0, 8, st));
            if (wide)
                k_owner_hist<K128><<<nblk, B, 0, st>>>(s->dkey.as<K128>(), n, nowners, nblk, bh, own, oid,
                                                       s->dfc.as<unsigned long long>(), s->dft.as<unsigned long long>(),
                                                       evmax);
            else
                k_owner_hist<unsigned long long><<<nblk, B, 0, st>>>(s->dkey.as<unsigned long long>(), n, nowners, nblk,
                                                                    bh, own, oid, s->dfc.as<unsigned long long>(),
                                                                    s->dft.as<unsigned long long>(), evmax);
            EC_CHECK(scan_incl_u32(s, bh, bhi, nbh));
            EC_CHECK(d2h(s, s->own_hi.data(), bhi, nbh * 4 + 8, st));  // (+ the event maxima)
        }
        if (compact && n) EC_CHECK(host_sync(s, st));  // (the event widths choose the record format)
    }
    int lfb = -1;  // compact records: bits of the window position (the read id above them), else full
    if (compact && lf_bits) {
        const unsigned int mr = n ? s->own_hi[nbh] : 0u, ml = n ? s->own_hi[nbh + 1] : 0u;
        int lb = 1, rb = 0;
        while (lb < 31 && (ml >> lb)) lb++;
        while (rb < 32 && (mr >> rb)) rb++;
        // (the all-ones code is "no event": it must stay out of range)
        if (lb + rb <= 32 && !(lb + rb == 32 && mr == (0xFFFFFFFFu >> lb) && ml == (1u << lb) - 1)) lfb = lb;
        *lf_bits = lfb;
    }
    if (n && d_out && lfb >= 0) {  // compact records (shard-relative events)
        if (wide)
            k_owner_scatter_c<K128><<<nblk, B, 0, st>>>(s->dkey.as<K128>(), s->dcnt.as<unsigned int>(),
                                                        s->dfc.as<unsigned long long>(), s->dft.as<unsigned long long>(),
                                                        n, nowners, nblk, bhi, reinterpret_cast<CRecW *>(d_out), lfb, oid);
        else
            k_owner_scatter_c<unsigned long long><<<nblk, B, 0, st>>>(
                s->dkey.as<unsigned long long>(), s->dcnt.as<unsigned int>(), s->dfc.as<unsigned long long>(),
                s->dft.as<unsigned long long>(), n, nowners, nblk, bhi, reinterpret_cast<CRec *>(d_out), lfb, oid);
    } else if (n && d_out) {  // the scatter is queued before the host waits for the owner counts
        if (wide)
            k_owner_scatter<K128><<<nblk, B, 0, st>>>(s->dkey.as<K128>(), s->dcnt.as<unsigned int>(),
                                                      s->dfc.as<unsigned long long>(), s->dft.as<unsigned long long>(),
                                                      n, nowners, nblk, bhi, reinterpret_cast<AggW *>(d_out),
                                                      s->shard_base << 32, oid);
        else
            k_owner_scatter<unsigned long long><<<nblk, B, 0, st>>>(
                s->dkey.as<unsigned long long>(), s->dcnt.as<unsigned int>(), s->dfc.as<unsigned long long>(),
                s->dft.as<unsigned long long>(), n, nowners, nblk, bhi, reinterpret_cast<Agg *>(d_out),
                s->shard_base << 32, oid);
    }
    EC_CHECK(host_sync(s, st));
    s->own_valid = true, s->own_rule = s->owner_rule, s->own_nowners = nowners, s->own_n = n, s->own_nblk = nblk;
    unsigned long long prev = 0;
    for (int i = 0; i < nowners; i++) {
        const unsigned long long end = n ? s->own_hi[(size_t)(i + 1) * nblk - 1] : 0ull;
        owner_counts[i] = end - prev;
        prev = end;
    }
    return EC_OK;
}

}  // extern "C"

// the owner merge; xin: k <= 32 records read in place (decode: the decoded copy, for the HBM table)
int merge_owned_impl(ec_session *s, const void *d_records, uint64_t n, int k, int limit, unsigned flags,
                     const XIn *xin = nullptr, const std::function<int(const Agg *&)> &decode = nullptr) {
    if (!s || (n && !d_records)) {
        set_error("null argument");
        return EC_ERR_ARG;
    }
    EC_CHECK(begin_call(s, k, flags));
    unsigned int U = 0;
    s->no_index = true;
    int rc = EC_OK;
    if (k > 32) {
        SolidIndexW sidx{};
        rc = phase_merge_w(s, reinterpret_cast<const AggW *>(d_records), n, (long long)limit, U, sidx);
    } else {
        SolidIndex sidx{};
        rc = phase_merge(s, reinterpret_cast<const Agg *>(d_records), n, (long long)limit, U, sidx, xin, decode);
    }
    s->no_index = false;
    EC_CHECK(rc);
    s->n_dense = U;
    collect_timing(s);
    s->stats_ok = true;
    return EC_OK;
}

extern "C" {

int ec_merge_owned(ec_session *s, const void *d_records, uint64_t n, int k, int limit, unsigned flags) {
    return merge_owned_impl(s, d_records, n, k, limit, flags);
}

// the merge of records received from nsrc ranks (ec_export_by_owner_ex: compact or full per
// source) -- decoded to exchange records with global events, then ec_merge_owned
int ec_merge_owned_from(ec_session *s, const void *d_records, int nsrc, const uint64_t *src_bytes,
                        const int64_t *src_read_base, const int32_t *src_lf_bits, int k, int limit, unsigned flags) {
    if (!s || nsrc < 1 || nsrc > MAX_OWNERS || !src_bytes || !src_read_base || !src_lf_bits || k < 1 || k > EC_MAX_K) {
        set_error("ec_merge_owned_from: bad arguments");
        return EC_ERR_ARG;
    }
    const size_t full = k > 32 ? sizeof(AggW) : sizeof(Agg), comp = k > 32 ? sizeof(CRecW) : sizeof(CRec);
    std::vector<unsigned long long> hoff(2 * (size_t)nsrc + 2);
    std::vector<long long> hb(nsrc);
    std::vector<int> hl(nsrc);
    unsigned long long bsum = 0, rsum = 0;
    for (int q = 0; q < nsrc; q++) {
        const size_t rb = src_lf_bits[q] >= 0 ? comp : full;
        if (src_bytes[q] % rb || src_lf_bits[q] > 31) {
            set_error("ec_merge_owned_from: source %d sends %llu bytes of %zu-B records", q,
                      (unsigned long long)src_bytes[q], rb);
            return EC_ERR_ARG;
        }
        hoff[q] = bsum;
        hoff[nsrc + 1 + q] = rsum;
        bsum += src_bytes[q];
        rsum += src_bytes[q] / rb;
        hb[q] = src_read_base[q];
        hl[q] = src_lf_bits[q];
    }
    hoff[nsrc] = bsum;
    hoff[2 * (size_t)nsrc + 1] = rsum;
    if (bsum && !d_records) {
        set_error("null records");
        return EC_ERR_ARG;
    }
    EC_HIP(hipSetDevice(s->device));
    hipStream_t st = s->stream;
    const size_t mbytes = hoff.size() * 8 + (size_t)nsrc * 12;
    EC_CHECK(s->xrec.ensure(std::max<uint64_t>(rsum, 1) * full + mbytes + 64));
    uint8_t *meta = s->xrec.as<uint8_t>() + std::max<uint64_t>(rsum, 1) * full;
    unsigned long long *doff = reinterpret_cast<unsigned long long *>(meta);
    long long *dbase = reinterpret_cast<long long *>(doff + hoff.size());
    int *dlfb = reinterpret_cast<int *>(dbase + nsrc);
    // one H2D copy from page-locked staging (three pageable copies cost ~0.1 ms a call)
    EC_HIP(hipStreamSynchronize(st));  // (the staging of an earlier call has been read)
    EC_CHECK(s->hmeta.resize(mbytes));
    memcpy(s->hmeta.data(), hoff.data(), hoff.size() * 8);
    memcpy(s->hmeta.data() + hoff.size() * 8, hb.data(), (size_t)nsrc * 8);
    memcpy(s->hmeta.data() + hoff.size() * 8 + (size_t)nsrc * 8, hl.data(), (size_t)nsrc * 4);
    EC_HIP(hipMemcpyAsync(doff, s->hmeta.data(), mbytes, hipMemcpyHostToDevice, st));
    if (k <= 32 && rsum && !kn().merge_decode) {
        // k <= 32: the merge reads the received records in place; the decoded copy only for the
        // HBM-table fallback (a bucket past its LDS table, or EC_FLAG_GENERAL)
        const XIn xin{static_cast<const uint8_t *>(d_records), doff, doff + nsrc + 1, dbase, dlfb, nsrc};
        auto decode = [&](const Agg *&out) -> int {
            k_uncompact<unsigned long long><<<grid_for(rsum, 256), 256, 0, s->stream>>>(
                static_cast<const uint8_t *>(d_records), doff, doff + nsrc + 1, dbase, dlfb, nsrc, rsum, s->xrec.as<Agg>());
            out = s->xrec.as<Agg>();
            return EC_OK;
        };
        return merge_owned_impl(s, s->xrec.p, rsum, k, limit, flags, &xin, decode);
    }
    if (rsum) {
        if (k > 32)
            k_uncompact<K128><<<grid_for(rsum, 256), 256, 0, st>>>(static_cast<const uint8_t *>(d_records), doff,
                                                                  doff + nsrc + 1, dbase, dlfb, nsrc, rsum,
                                                                  s->xrec.as<AggW>());
        else
            k_uncompact<unsigned long long><<<grid_for(rsum, 256), 256, 0, st>>>(
                static_cast<const uint8_t *>(d_records), doff, doff + nsrc + 1, dbase, dlfb, nsrc, rsum, s->xrec.as<Agg>());
    }
    return ec_merge_owned(s, s->xrec.p, rsum, k, limit, flags);
}

int ec_compact_record_bytes(int k) { return k > 32 ? (int)sizeof(CRecW) : (int)sizeof(CRec); }

int ec_export_dense(ec_session *s, void *d_out) {
    if (!s) return EC_ERR_ARG;
    EC_HIP(hipSetDevice(s->device));
    const unsigned int n = s->n_dense;
    if (n && d_out) {
        if (s->k > 32)
            k_export_dense<K128><<<grid_for(n, 256), 256, 0, s->stream>>>(
                s->dkey.as<K128>(), s->dcnt.as<unsigned int>(), s->dfc.as<unsigned long long>(),
                s->dft.as<unsigned long long>(), n, reinterpret_cast<AggW *>(d_out), s->shard_base << 32);
        else
            k_export_dense<unsigned long long><<<grid_for(n, 256), 256, 0, s->stream>>>(
                s->dkey.as<unsigned long long>(), s->dcnt.as<unsigned int>(), s->dfc.as<unsigned long long>(),
                s->dft.as<unsigned long long>(), n, reinterpret_cast<Agg *>(d_out), s->shard_base << 32);
        EC_CHECK(host_sync(s, s->stream));
    }
    return EC_OK;
}

uint64_t ec_dense_count(ec_session *s) { return s ? s->n_dense : 0; }

int ec_merge_owned_export(ec_session *s, const void *d_records, uint64_t n, int k, int limit, unsigned flags,
                          void *d_out) {
    EC_CHECK(ec_merge_owned(s, d_records, n, k, limit, flags));
    return ec_export_dense(s, d_out);
}

int ec_assemble_from_solid(ec_session *s, const void *d_records, uint64_t n, int k, unsigned flags) {
    if (!s || (n && !d_records)) {
        set_error("null argument");
        return EC_ERR_ARG;
    }
    EC_CHECK(begin_call(s, k, flags));
    unsigned int U = 0;
    if (k > 32) {
        SolidIndexW sidx{};
        EC_CHECK(phase_merge_w(s, reinterpret_cast<const AggW *>(d_records), n, LLONG_MIN, U, sidx));
        return phase_graph<OpsW>(s, k, U, sidx);
    }
    // the gathered keys are distinct; the bucketed merge (sort by bucket + LDS tables) is also
    // the fastest loader: measured 0.42 ms at 4.6 M keys against 0.60 ms for per-key CAS
    // inserts into the HBM sub-table (random-address atomics)
    SolidIndex sidx{};
    EC_CHECK(phase_merge(s, reinterpret_cast<const Agg *>(d_records), n, LLONG_MIN, U, sidx));
    return phase_graph<Ops64>(s, k, U, sidx);
}

int ec_record_bytes(int k) { return k > 32 ? (int)sizeof(AggW) : (int)sizeof(Agg); }

int ec_graph_load(ec_session *s, const void *d_records, uint64_t n, int k, unsigned flags) {
    if (!s || (n && !d_records)) {
        set_error("null argument");
        return EC_ERR_ARG;
    }
    s->graph_loaded = false;
    // the owner merge's bucket marks (this rank's segment of the set loaded here) outlive the load
    const uint64_t marks = s->seg_marks;
    EC_CHECK(begin_call(s, k, flags));
    s->seg_marks = marks;
    unsigned int U = 0;
    if (k > 32)
        EC_CHECK(phase_load_det_w(s, reinterpret_cast<const AggW *>(d_records), n, U, s->gidxw));
    else
        EC_CHECK(phase_load_det(s, reinterpret_cast<const Agg *>(d_records), n, U, s->gidx));
    if (2ull * U >= (unsigned long long)CYC) {
        set_error("too many solid k-mers (%u) for 31-bit node ids", U);
        return EC_ERR_CAPACITY;
    }
    s->n_dense = U;
    s->graph_loaded = true;
    collect_timing(s);
    s->stats_ok = true;
    return EC_OK;
}

int ec_graph_links_part(ec_session *s, uint64_t lo, uint64_t hi, uint32_t *d_succ) {
    refresh_knobs();
    if (!s || !s->graph_loaded || lo > hi || hi > s->n_dense || (hi > lo && !d_succ)) {
        set_error("ec_graph_links_part: no loaded solid set or bad range [%llu, %llu)", (unsigned long long)lo,
                  (unsigned long long)hi);
        return EC_ERR_ARG;
    }
    EC_HIP(hipSetDevice(s->device));
    if (hi > lo) {
        const uint64_t n = 2 * (hi - lo);
        if (s->k > 32)
            k_links_part<OpsW, SolidIndexW><<<grid_for(n, 256), 256, 0, s->stream>>>(
                s->gidxw, s->dkey.as<K128>(), (unsigned int)lo, (unsigned int)hi, s->k, d_succ);
        else
            k_links_part<Ops64, SolidIndex><<<grid_for(n, 256), 256, 0, s->stream>>>(
                s->gidx, s->dkey.as<unsigned long long>(), (unsigned int)lo, (unsigned int)hi, s->k, d_succ);
        EC_HIP(hipGetLastError());
    }
    EC_CHECK(host_sync(s, s->stream));
    return EC_OK;
}

int ec_graph_load_links(ec_session *s, const void *d_records, uint64_t n, int k, unsigned flags, uint64_t lo,
                        uint64_t hi, uint32_t *d_succ) {
    EC_CHECK(ec_graph_load(s, d_records, n, k, flags));
    return ec_graph_links_part(s, lo, hi, d_succ);
}

int ec_graph_finish(ec_session *s, const uint32_t *d_succ, unsigned flags) {
    if (!s || !s->graph_loaded || s->placed || (s->n_dense && !d_succ)) {
        set_error("ec_graph_finish: no loaded solid set");
        return EC_ERR_ARG;
    }
    const unsigned int U = (unsigned int)s->n_dense;
    const ec_stats keep = s->stats;
    EC_CHECK(begin_call(s, s->k, flags));
    s->stats = keep;
    for (float &v : s->stats.stage_ms) v = 0.0f;
    for (float &v : s->stats.kernel_ms) v = 0.0f;
    s->graph_loaded = false;
    if (s->k > 32) return phase_graph<OpsW>(s, s->k, U, s->gidxw, d_succ);
    return phase_graph<Ops64>(s, s->k, U, s->gidx, d_succ);
}

// multi-GPU partitioned finish (see part_chains above); include/eulerhip.h
int ec_graph_chains_part(ec_session *s, uint64_t lo, uint64_t hi, const uint32_t *d_succ, void *d_super,
                         uint64_t *n_super) {
    refresh_knobs();
    if (!s || !s->graph_loaded || lo > hi || hi > s->n_dense || !n_super ||
        (hi > lo && !d_succ && !s->placed) ||
        (s->placed && (lo != s->seg_lo || hi != s->seg_lo + s->seg_Ur))) {
        set_error("ec_graph_chains_part: no loaded solid set or bad range [%llu, %llu)", (unsigned long long)lo,
                  (unsigned long long)hi);
        return EC_ERR_ARG;
    }
    EC_HIP(hipSetDevice(s->device));
    SuperRec *out = static_cast<SuperRec *>(d_super);
    return s->k > 32 ? part_chains<OpsW>(s, lo, hi, d_succ, out, n_super)
                     : part_chains<Ops64>(s, lo, hi, d_succ, out, n_super);
}

int ec_graph_rank_supers(ec_session *s, const void *d_supers, uint64_t n) {
    if (!s || !s->graph_loaded || (n && !d_supers)) {
        set_error("ec_graph_rank_supers: no loaded solid set");
        return EC_ERR_ARG;
    }
    EC_HIP(hipSetDevice(s->device));
    return part_rank(s, static_cast<const SuperRec *>(d_supers), n);
}

int ec_graph_starts_part(ec_session *s, int have_supers, void *d_starts, uint64_t *n_starts) {
    if (!s || !s->graph_loaded || !n_starts) {
        set_error("ec_graph_starts_part: no loaded solid set");
        return EC_ERR_ARG;
    }
    EC_HIP(hipSetDevice(s->device));
    return part_starts(s, have_supers != 0, static_cast<StartRec *>(d_starts), n_starts);
}

// the records a step called with a NULL output counted (exact-size buffers)
static int take_pending(ec_session *s, int kind, const void *d_out, const char *what, uint64_t &n) {
    if (!s || s->hold.kind != kind || (s->hold.n && !d_out)) {
        set_error("%s: no pending records of this step (call it with a NULL output first)", what);
        return EC_ERR_STATE;
    }
    n = s->hold.n;
    s->hold.kind = 0;
    return hipSetDevice(s->device) == hipSuccess ? EC_OK : EC_ERR_HIP;
}

int ec_graph_place_copy(ec_session *s, void *d_jrecs) {
    uint64_t n = 0;
    EC_CHECK(take_pending(s, 1, d_jrecs, "ec_graph_place_copy", n));
    if (n) {
        if (s->k > 32)
            k_gather_recs<RecJ><<<grid_for(n, 256), 256, 0, s->stream>>>(s->jrec.as<RecJ>(), s->midx2.as<unsigned int>(), n,
                                                                      static_cast<RecJ *>(d_jrecs));
        else
            k_gather_recs<RecJ64><<<grid_for(n, 256), 256, 0, s->stream>>>(
                s->jrec.as<RecJ64>(), s->midx2.as<unsigned int>(), n, static_cast<RecJ64 *>(d_jrecs));
    }
    return host_sync(s, s->stream);
}

int ec_graph_chains_copy(ec_session *s, void *d_super) {
    uint64_t n = 0;
    EC_CHECK(take_pending(s, 2, d_super, "ec_graph_chains_copy", n));
    return part_chains_copy(s, n, s->hold.ntiles, s->hold.planned, static_cast<SuperRec *>(d_super));
}

int ec_graph_starts_copy(ec_session *s, void *d_starts) {
    uint64_t n = 0;
    EC_CHECK(take_pending(s, 3, d_starts, "ec_graph_starts_copy", n));
    return part_starts_copy(s, n, static_cast<StartRec *>(d_starts));
}

int ec_graph_layout(ec_session *s, const void *d_starts, uint64_t n, uint64_t *n_chars) {
    if (!s || !s->graph_loaded || !n_chars || (n && !d_starts)) {
        set_error("ec_graph_layout: no loaded solid set");
        return EC_ERR_ARG;
    }
    EC_HIP(hipSetDevice(s->device));
    return part_layout(s, static_cast<const StartRec *>(d_starts), n, n_chars);
}

int ec_graph_emit_part(ec_session *s, char *d_chars, void *d_ends) {
    if (!s || !s->graph_loaded || (s->seg_nchars && !d_chars) || (s->seg_nc && !d_ends)) {
        set_error("ec_graph_emit_part: no layout");
        return EC_ERR_ARG;
    }
    EC_HIP(hipSetDevice(s->device));
    return s->k > 32 ? part_emit<OpsW>(s, d_chars, d_ends) : part_emit<Ops64>(s, d_chars, d_ends);
}

int ec_graph_collect(ec_session *s, const char *d_chars, const void *d_ends, uint64_t n_pal) {
    if (!s || !s->graph_loaded || (s->seg_nchars && !d_chars) || (s->seg_nc && !d_ends) || 2 * n_pal > 2 * s->n_dense) {
        set_error("ec_graph_collect: no layout");
        return EC_ERR_ARG;
    }
    EC_HIP(hipSetDevice(s->device));
    return s->k > 32 ? part_collect<OpsW>(s, d_chars, d_ends, n_pal) : part_collect<Ops64>(s, d_chars, d_ends, n_pal);
}

int ec_graph_emit_runs(ec_session *s, uint64_t *nbytes) {
    if (!s || !s->graph_loaded || !nbytes) {
        set_error("ec_graph_emit_runs: no layout");
        return EC_ERR_ARG;
    }
    EC_HIP(hipSetDevice(s->device));
    return s->k > 32 ? part_emit_runs<OpsW>(s, nbytes) : part_emit_runs<Ops64>(s, nbytes);
}

int ec_graph_copy_runs(ec_session *s, void *d_out) {
    if (!s || !s->runs_ready || !d_out) {
        set_error("ec_graph_copy_runs: no emitted runs (ec_graph_emit_runs)");
        return EC_ERR_ARG;
    }
    EC_HIP(hipSetDevice(s->device));
    return s->k > 32 ? part_copy_runs<OpsW>(s, d_out) : part_copy_runs<Ops64>(s, d_out);
}

int ec_graph_collect_runs(ec_session *s, const void *d_in, int nsrc, const uint64_t *src_bytes, uint64_t n_pal) {
    if (!s || !s->graph_loaded || nsrc < 1 || !src_bytes || !d_in || n_pal > s->n_dense) {
        set_error("ec_graph_collect_runs: no layout or bad arguments");
        return EC_ERR_ARG;
    }
    EC_HIP(hipSetDevice(s->device));
    return s->k > 32 ? part_collect_runs<OpsW>(s, static_cast<const uint8_t *>(d_in), nsrc, src_bytes, n_pal)
                     : part_collect_runs<Ops64>(s, static_cast<const uint8_t *>(d_in), nsrc, src_bytes, n_pal);
}

int ec_end_record_bytes(int k) { return k > 32 ? 16 : 8; }
int ec_junction_record_bytes(int k) { return k > 32 ? (int)sizeof(RecJ) : (int)sizeof(RecJ64); }
int ec_link_record_bytes(void) { return (int)sizeof(LinkRec); }

}  // extern "C"

// ---- junction-partitioned graph (junction.h) ------------------------------------------------
// counting sort of n ids (bins 0..nbins-1) -> perm (midx2) and bin starts bstart[0..nbins]
int bin_sort(ec_session *s, const unsigned int *bid, uint64_t n, unsigned int nbins, unsigned long long *bstart) {
    EC_CHECK(s->midx2.ensure(std::max<uint64_t>(n, 1) * 4));
    if (!n) {
        EC_HIP(hipMemsetAsync(bstart, 0, (nbins + 1ull) * 8, s->stream));
        return EC_OK;
    }
    return cs_sort(s, bid, n, nbins, bstart, true);
}

template <typename K>
int graph_place(ec_session *s, uint64_t lo, uint64_t U, int nowners, void *d_out, uint64_t *owner_counts,
                uint64_t *n_pal) {
    using R = typename JRecOf<K>::R;
    using Ops = typename std::conditional<sizeof(K) == 8, Ops64, OpsW>::type;
    hipStream_t st = s->stream;
    const unsigned B = 256;
    Scalars *dsc = s->scal.as<Scalars>();
    const uint64_t Ur = s->n_dense, Uu = std::max<uint64_t>(U, 1);
    // the merge's dense arrays [0, Ur) -> global ids [lo, lo + Ur) of U-sized arrays
    EC_CHECK(s->recs.ensure(std::max<uint64_t>(Ur, 1) * sizeof(K)));
    EC_CHECK(s->recs2.ensure(std::max<uint64_t>(Ur, 1) * 16));
    EC_CHECK(s->midx.ensure(std::max<uint64_t>(Ur, 1) * 4));
    unsigned long long *tfc = s->recs2.as<unsigned long long>(), *tft = tfc + Ur;
    if (Ur) {
        EC_HIP(hipMemcpyAsync(s->recs.p, s->dkey.p, Ur * sizeof(K), hipMemcpyDeviceToDevice, st));
        EC_HIP(hipMemcpyAsync(s->midx.p, s->dcnt.p, Ur * 4, hipMemcpyDeviceToDevice, st));
        EC_HIP(hipMemcpyAsync(tfc, s->dfc.p, Ur * 8, hipMemcpyDeviceToDevice, st));
        EC_HIP(hipMemcpyAsync(tft, s->dft.p, Ur * 8, hipMemcpyDeviceToDevice, st));
    }
    if (s->dkey.cap < Uu * sizeof(K) || s->dcnt.cap < Uu * 4 || s->dfc.cap < Uu * 8 || s->dft.cap < Uu * 8)
        EC_HIP(hipStreamSynchronize(st));  // (the ensure()s below free the copies' sources)
    EC_CHECK(s->dkey.ensure(Uu * sizeof(K)));
    EC_CHECK(s->dcnt.ensure(Uu * 4));
    EC_CHECK(s->dfc.ensure(Uu * 8));
    EC_CHECK(s->dft.ensure(Uu * 8));
    EC_CHECK(s->upal.ensure(Uu));
    EC_CHECK(s->succ.ensure(2 * Uu * 4));
    if (Ur) {
        EC_HIP(hipMemcpyAsync(s->dkey.as<K>() + lo, s->recs.p, Ur * sizeof(K), hipMemcpyDeviceToDevice, st));
        EC_HIP(hipMemcpyAsync(s->dcnt.as<unsigned int>() + lo, s->midx.p, Ur * 4, hipMemcpyDeviceToDevice, st));
        EC_HIP(hipMemcpyAsync(s->dfc.as<unsigned long long>() + lo, tfc, Ur * 8, hipMemcpyDeviceToDevice, st));
        EC_HIP(hipMemcpyAsync(s->dft.as<unsigned long long>() + lo, tft, Ur * 8, hipMemcpyDeviceToDevice, st));
        EC_HIP(hipMemsetAsync(s->succ.as<unsigned int>() + 2 * lo, 0xFF, 2 * Ur * 4, st));
    }
    EC_HIP(hipMemsetAsync(&dsc->npal, 0, 4, st));
    if (Ur)
        EC_CHECK(launch_upal<Ops>(st, s->dkey.as<K>() + lo, (unsigned int)Ur, s->k, s->upal.as<uint8_t>() + lo,
                                  &dsc->npal));
    // junction records routed to the junctions' owners (the keys' rule, shard.h OwnerFn)
    OwnerFn own = owner_fn(s->k);
    if (s->owner_rule == 1) own.sk = 0, own.wk = 0;
    JOwnerFn jown{};
    jown.sk = own.sk;
    if (own.sk) jown.mcj = sk_cfg(s->k - 1);
    jown.wj = own.wk ? s->k - 1 : 0;
    const uint64_t nslot = 4 * Ur;
    EC_CHECK(s->jrec.ensure(std::max<uint64_t>(nslot, 1) * sizeof(R)));
    EC_CHECK(s->joid.ensure(std::max<uint64_t>(nslot, 1) * 4));
    EC_CHECK(s->jseg.ensure(((size_t)nowners + 2) * 8));
    unsigned long long *ostart = s->jseg.as<unsigned long long>();
    if (Ur)
        k_junction_emit<K><<<grid_for(Ur, B), B, 0, st>>>(s->dkey.as<K>(), s->upal.as<uint8_t>(), (unsigned int)lo,
                                                         (unsigned int)Ur, s->k, jown, (unsigned int)nowners,
                                                         s->jrec.as<R>(), s->joid.as<unsigned int>());
    // owner-major order: counting sort by owner (NONE slots in the last bin, dropped)
    EC_CHECK(s->joid.ensure(std::max<uint64_t>(nslot, 1) * 4));
    if (nslot) k_none_to_bin<<<grid_for(nslot, B), B, 0, st>>>(s->joid.as<unsigned int>(), nslot, (unsigned int)nowners);
    EC_CHECK(bin_sort(s, s->joid.as<unsigned int>(), nslot, (unsigned int)nowners + 1, ostart));
    if (nslot && d_out)  // (NULL: counted only, ec_graph_place_copy gathers the owned records)
        k_gather_recs<R><<<grid_for(nslot, B), B, 0, st>>>(s->jrec.as<R>(), s->midx2.as<unsigned int>(), nslot,
                                                          static_cast<R *>(d_out));
    std::vector<unsigned long long> hs((size_t)nowners + 2);
    EC_CHECK(d2h(s, hs.data(), ostart, ((size_t)nowners + 2) * 8, st));
    unsigned int npal = 0;
    EC_CHECK(d2h(s, &npal, &dsc->npal, 4, st));
    EC_CHECK(host_sync(s, st));
    for (int r = 0; r < nowners; r++) owner_counts[r] = hs[r + 1] - hs[r];
    if (!d_out) s->hold = ec_session::Pending{1, hs[nowners], 0, false};
    *n_pal = npal;
    s->seg_lo = lo;
    s->seg_Ur = Ur;
    s->n_dense = (unsigned int)U;
    s->placed = true;
    s->graph_loaded = true;  // (the part_* steps' state: the placed segment)
    s->seg_n0 = 2 * lo;
    s->seg_n1 = 2 * (lo + Ur);
    return EC_OK;
}

// bin starts of n bin ids sorted ascending (bstart[b] = first index with id >= b, bstart[nb] = n)
__global__ void __launch_bounds__(256) k_sorted_starts(const unsigned int *key, uint64_t n, unsigned int nb,
                                                      unsigned long long *bstart) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned int kk = key[i];
        const long long prev = i ? (long long)key[i - 1] : -1ll;
        for (long long b = prev + 1; b <= (long long)kk; b++) bstart[b] = i;
        if (i + 1 == n)
            for (long long b = (long long)kk + 1; b <= (long long)nb; b++) bstart[b] = n;
    }
}
__global__ void __launch_bounds__(256) k_iota_u32(unsigned int *v, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        v[i] = (unsigned int)i;
}

template <typename R>
int graph_join(ec_session *s, const R *d_recs, uint64_t n, int nowners, const uint64_t *seg_lo, LinkRec *d_links,
               uint64_t *owner_counts) {
    hipStream_t st = s->stream;
    const unsigned B = 256;
    s->hold.kind = 0;
    constexpr int BT_CS = 14, BT_MAX = 22;  // counting sort's LDS histogram limit; radix sort past it
    EC_CHECK(s->jseg.ensure(((size_t)nowners + 2) * 8 + ((size_t)(1u << BT_MAX) + 1) * 8 + 64));
    unsigned long long *dseg = s->jseg.as<unsigned long long>();
    unsigned long long *bstart = dseg + nowners + 2;
    EC_HIP(hipMemcpyAsync(dseg, seg_lo, ((size_t)nowners + 1) * 8, hipMemcpyHostToDevice, st));
    EC_CHECK(s->jcnt.ensure(16));
    unsigned int *flag = s->jcnt.as<unsigned int>(), *nout = flag + 1;
    EC_CHECK(s->jout.ensure(std::max<uint64_t>(n, 1) * sizeof(LinkRec)));
    LinkRec *outbox = s->jout.as<LinkRec>();
    // join buckets: ~n / 2 junction groups, <= ~900 a 2048-slot table; up to 2^14 buckets by the
    // counting sort (its LDS histogram's limit), up to 2^22 by a radix sort of the bucket ids --
    // sub-buckets (each re-reading its bucket's records) only past that or when forced: config 5's
    // per-rank step joined 4e8 records in 2^14 buckets x 16 sub-buckets in 195 ms.  A table that
    // overflows (skewed junction hashes) retries with 4096 slots, then finer buckets, then more
    // sub-buckets (EULERHIP_JUNCTION_BT / _SB / _CLAIM force the split / a smaller claim cap)
    const int btmax = kn().junction_bt >= 0 ? std::min(kn().junction_bt, BT_MAX) : BT_MAX;
    const double groups = (double)n / 2.0;
    int bt = 0, sb = 0;
    while (bt < btmax && groups / (double)(1ull << bt) > 900.0) bt++;
    while (sb < 8 && groups / (double)(1ull << (bt + sb)) > 900.0) sb++;
    if (kn().junction_sb > sb) sb = std::min(kn().junction_sb, 8);
    bool big = groups / (double)(1ull << (bt + sb)) > 1500.0;
    for (;;) {
        const unsigned int nb = 1u << bt;
        const unsigned int claim = kn().junction_claim > 0 ? (unsigned int)kn().junction_claim
                                                           : (big ? 4096u : 2048u) - 1u;
        EC_CHECK(s->joid.ensure(std::max<uint64_t>(n, 1) * 4));
        EC_HIP(hipMemsetAsync(flag, 0, 8, st));
        if (n) k_junction_bucket<R><<<grid_for(n, B), B, 0, st>>>(d_recs, n, bt, s->joid.as<unsigned int>());
        if ((bt <= BT_CS && kn().junction_radix != 1) || !n) {
            EC_CHECK(bin_sort(s, s->joid.as<unsigned int>(), n, nb, bstart));
        } else {  // record order by bucket id: rocprim radix sort of (id, index) pairs over bt bits
            EC_CHECK(s->mbid.ensure(n * 4));
            EC_CHECK(s->mbid2.ensure(n * 4));
            EC_CHECK(s->midx2.ensure(n * 4));
            k_iota_u32<<<grid_for(n, B, 8192), B, 0, st>>>(s->mbid.as<unsigned int>(), n);
            size_t bytes = 0;
            EC_HIP(rocprim::radix_sort_pairs(nullptr, bytes, s->joid.as<unsigned int>(), s->mbid2.as<unsigned int>(),
                                             s->mbid.as<unsigned int>(), s->midx2.as<unsigned int>(), (size_t)n, 0, bt,
                                             st));
            EC_CHECK(s->tmp.ensure(bytes));
            EC_HIP(rocprim::radix_sort_pairs(s->tmp.p, bytes, s->joid.as<unsigned int>(), s->mbid2.as<unsigned int>(),
                                             s->mbid.as<unsigned int>(), s->midx2.as<unsigned int>(), (size_t)n, 0, bt,
                                             st));
            k_sorted_starts<<<grid_for(n, B, 8192), B, 0, st>>>(s->mbid2.as<unsigned int>(), n, nb, bstart);
        }
        const unsigned int n0 = (unsigned int)(2 * s->seg_lo), n1 = (unsigned int)(2 * (s->seg_lo + s->seg_Ur));
        if (n) {
            if (big)
                k_junction_join<4096, 512, R><<<nb, 512, 0, st>>>(d_recs, s->midx2.as<unsigned int>(), bstart, n0, n1,
                                                                  s->succ.as<unsigned int>(), outbox, nout,
                                                                  (unsigned int)n, flag, bt, sb, claim);
            else
                k_junction_join<2048, 512, R><<<nb, 512, 0, st>>>(d_recs, s->midx2.as<unsigned int>(), bstart, n0, n1,
                                                                  s->succ.as<unsigned int>(), outbox, nout,
                                                                  (unsigned int)n, flag, bt, sb, claim);
            EC_HIP(hipGetLastError());
        }
        // outbox -> destination-major link records, sized by n on the host (the count stays on
        // the device: one read-back for the flags and the destinations' counts)
        if (n) {
            k_link_dest<<<grid_for(n, B), B, 0, st>>>(outbox, nout, (unsigned int)n, dseg, (unsigned int)nowners,
                                                      s->joid.as<unsigned int>());
            EC_CHECK(bin_sort(s, s->joid.as<unsigned int>(), n, (unsigned int)nowners + 1, bstart));
            k_gather_recs<LinkRec><<<grid_for(n, B), B, 0, st>>>(outbox, s->midx2.as<unsigned int>(), n, d_links);
        } else {
            EC_HIP(hipMemsetAsync(bstart, 0, ((size_t)nowners + 2) * 8, st));
        }
        unsigned int hf[2] = {0, 0};
        std::vector<unsigned long long> hs((size_t)nowners + 2);
        EC_CHECK(d2h(s, hf, flag, 8, st));
        EC_CHECK(d2h(s, hs.data(), bstart, ((size_t)nowners + 2) * 8, st));
        EC_CHECK(host_sync(s, st));
        if (hf[0] & 2u) {
            set_error("junction join: link outbox overflow");
            return EC_ERR_STATE;
        }
        if (hf[0] & 1u) {  // a table past its slots: bigger tables, finer buckets, more sub-buckets
            // (succ: a failed attempt's local links are the same links the retry writes)
            if (!big) big = true;
            else if (bt < btmax) bt++;
            else if (sb < 8) sb++;
            else {
                set_error("junction join: a bucket of %llu records overflows its table at 2^%d x 2^%d buckets",
                          (unsigned long long)n, bt, sb);
                return EC_ERR_CAPACITY;
            }
            s->stats.table_retries++;
            continue;
        }
        for (int r = 0; r < nowners; r++) owner_counts[r] = hs[r + 1] - hs[r];
        return EC_OK;
    }
}

extern "C" {

int ec_graph_place(ec_session *s, uint64_t lo, uint64_t U, int nowners, void *d_jrecs, uint64_t *owner_counts,
                   uint64_t *n_pal) {
    refresh_knobs();
    if (!s || nowners < 1 || nowners > MAX_OWNERS || !owner_counts || !n_pal || lo + s->n_dense > U ||
        2 * U >= (uint64_t)CYC) {
        set_error("ec_graph_place: bad arguments (segment [%llu, +%u) of %llu ids)", (unsigned long long)lo,
                  s ? s->n_dense : 0u, (unsigned long long)U);
        return EC_ERR_ARG;
    }
    EC_HIP(hipSetDevice(s->device));
    return s->k > 32 ? graph_place<K128>(s, lo, U, nowners, d_jrecs, owner_counts, n_pal)
                     : graph_place<unsigned long long>(s, lo, U, nowners, d_jrecs, owner_counts, n_pal);
}

int ec_graph_join(ec_session *s, const void *d_jrecs, uint64_t n, int nowners, const uint64_t *seg_lo, void *d_links,
                  uint64_t *owner_counts) {
    if (!s || !s->placed || nowners < 1 || nowners > MAX_OWNERS || !seg_lo || !owner_counts ||
        (n && (!d_jrecs || !d_links))) {
        set_error("ec_graph_join: no placed segment or bad arguments");
        return EC_ERR_ARG;
    }
    for (int r = 0; r < nowners; r++)
        if (seg_lo[r] > seg_lo[r + 1] || seg_lo[nowners] != s->n_dense) {
            set_error("ec_graph_join: segment bounds not ascending up to %u", s->n_dense);
            return EC_ERR_ARG;
        }
    EC_HIP(hipSetDevice(s->device));
    return s->k > 32 ? graph_join<RecJ>(s, static_cast<const RecJ *>(d_jrecs), n, nowners, seg_lo,
                                        static_cast<LinkRec *>(d_links), owner_counts)
                     : graph_join<RecJ64>(s, static_cast<const RecJ64 *>(d_jrecs), n, nowners, seg_lo,
                                          static_cast<LinkRec *>(d_links), owner_counts);
}

int ec_graph_links_apply(ec_session *s, const void *d_links, uint64_t n) {
    if (!s || !s->placed || (n && !d_links)) {
        set_error("ec_graph_links_apply: no placed segment");
        return EC_ERR_ARG;
    }
    EC_HIP(hipSetDevice(s->device));
    hipStream_t st = s->stream;
    EC_CHECK(s->jcnt.ensure(16));
    unsigned int *bad = s->jcnt.as<unsigned int>();
    EC_HIP(hipMemsetAsync(bad, 0, 4, st));
    if (n)
        k_links_apply<<<grid_for(n, 256), 256, 0, st>>>(static_cast<const LinkRec *>(d_links), n,
                                                        (unsigned int)(2 * s->seg_lo),
                                                        (unsigned int)(2 * (s->seg_lo + s->seg_Ur)),
                                                        s->succ.as<unsigned int>(), bad);
    unsigned int hb = 0;
    EC_CHECK(d2h(s, &hb, bad, 4, st));
    EC_CHECK(host_sync(s, st));
    if (hb) {
        set_error("ec_graph_links_apply: a link record names a node outside this segment");
        return EC_ERR_ARG;
    }
    return EC_OK;
}

int ec_super_record_bytes(void) { return (int)sizeof(SuperRec); }
int ec_start_record_bytes(void) { return (int)sizeof(StartRec); }

int ec_assemble_from_kmers(ec_session *s, const char *kmers, const uint32_t *counts, uint64_t n, int k, unsigned flags) {
    if (!s || (n && (!kmers || !counts))) {
        set_error("null argument");
        return EC_ERR_ARG;
    }
    EC_CHECK(begin_call(s, k, flags));
    hipStream_t st = s->stream;
    EC_CHECK(s->dchars.ensure(std::max<size_t>(n * (size_t)k, 1)));
    EC_CHECK(s->dcounts.ensure(std::max<size_t>(n * 4, 4)));
    const bool wide = k > 32;
    EC_CHECK(s->recs2.ensure(std::max<size_t>(n * (wide ? sizeof(AggW) : sizeof(Agg)), 16)));
    Scalars *dsc = s->scal.as<Scalars>();
    if (n) {
        EC_HIP(hipMemcpyAsync(s->dchars.p, kmers, n * (size_t)k, hipMemcpyHostToDevice, st));
        EC_HIP(hipMemcpyAsync(s->dcounts.p, counts, n * 4, hipMemcpyHostToDevice, st));
        if (wide)
            k_kmers_to_agg<OpsW><<<grid_for(n, 256), 256, 0, st>>>(s->dchars.as<char>(), s->dcounts.as<unsigned int>(),
                                                                  n, k, s->recs2.as<AggW>(), &dsc->bad);
        else
            k_kmers_to_agg<Ops64><<<grid_for(n, 256), 256, 0, st>>>(s->dchars.as<char>(), s->dcounts.as<unsigned int>(),
                                                                   n, k, s->recs2.as<Agg>(), &dsc->bad);
        unsigned long long bad = 0;
        EC_CHECK(d2h(s, &bad, &dsc->bad, 8, st));
        EC_CHECK(host_sync(s, st));
        if (bad != ~0ull)  // bytes other than A/C/G/T: opaque symbols (extended.h)
            return assemble_kmers_extended(s, kmers, n, k);
    }
    unsigned int U = 0;
    if (wide) {
        SolidIndexW sidx{};
        EC_CHECK(phase_merge_w(s, s->recs2.as<AggW>(), n, LLONG_MIN, U, sidx));
        return phase_graph<OpsW>(s, k, U, sidx);
    }
    SolidIndex sidx{};
    EC_CHECK(phase_merge(s, s->recs2.as<Agg>(), n, LLONG_MIN, U, sidx));
    return phase_graph<Ops64>(s, k, U, sidx);
}

}  // extern "C"
