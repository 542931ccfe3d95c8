// ingest.cpp -- native read ingest: FASTA / FASTQ file -> one packed
// base buffer + uint64 offsets (CSR), the input layout of ec_assemble_* and ec_count_shard.
//
// Semantics follow the reference's readers:
//   EC_FASTA_RECORDS  one read per '>' record, sequence lines stripped and joined -- the
//                     SeqIO parse of tests/referenceAssembler.py:28, src/fastareader/parse_fasta.py:32-45
//                     and src/readTest.c:9-50 (text before the first header is ignored);
//   EC_FASTA_LINES    one read per non-header line, stripped (empty lines give empty reads) --
//                     read_fasta, src/eulercuda.py:437-445;
//   EC_FASTQ          the sequence line of every 4-line record -- read_fastq, src/eulercuda.py:43-55.
// "stripped" = leading / trailing ASCII whitespace removed (Python str.strip()).
//
// The file is memory-mapped and parsed by T threads over byte ranges in two passes (count,
// then copy at prefix-summed offsets), so a multi-GB read set is ingested at memory speed.
#include "common.h"

#include <hip/hip_runtime.h>

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#if defined(__SSE2__) && !defined(__HIP_DEVICE_COMPILE__)  // (host pass only)
#include <emmintrin.h>
#endif

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <chrono>
#include <mutex>
#include <thread>
#include <vector>

using ec::set_error;

struct ec_reads {
    std::vector<uint8_t> bases;
    std::vector<uint64_t> offsets;  // n_reads + 1
    // EC_READS_PACKED: the bases as 2-bit codes (4 a byte, ec_assemble_packed_host's layout) in
    // page-locked memory, the bytes other than A/C/G/T as exceptions; bases stays empty
    bool packed = false;
    uint8_t *codes = nullptr;
    uint64_t nbases = 0;
    uint32_t read_len = 0;  // every read this long (0: lengths differ)
    bool pinned = true;     // codes from hipHostMalloc (else malloc)
    size_t codes_cap = 0;
    std::vector<uint64_t> exc_pos;
    std::vector<uint8_t> exc_byte;
    int staged_dev = -1;    // device of the last ec_stage_packed_reads: its async H2D copy may still read codes
    ~ec_reads();
};

namespace {

inline bool is_ws(uint8_t c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\v' || c == '\f'; }

// [b, e) of line content after strip()
inline void strip(const uint8_t *p, uint64_t &b, uint64_t &e) {
    while (b < e && is_ws(p[b])) b++;
    while (e > b && is_ws(p[e - 1])) e--;
}

struct Chunk {
    uint64_t lo = 0, hi = 0;       // byte range [lo, hi), starts at a line start
    uint64_t lines_before = 0;     // FASTQ: global index of the first line of the chunk
    uint64_t reads = 0, bases = 0; // pass-1 counts
    uint64_t exc = 0;              // packed: bytes other than A/C/G/T among its bases
};

// 2-bit code of an ASCII base (A 0, C 1, G 2, T 3) and whether the byte is exactly that letter
inline uint8_t code2(uint8_t c) { return (uint8_t)(((c >> 1) ^ (c >> 2)) & 3u); }
inline bool is_exc(uint8_t c) {
    static const uint8_t letter[4] = {'A', 'C', 'G', 'T'};
    return letter[code2(c)] != c;
}
// SWAR over 8 bytes: 0x80 in every byte that is not exactly A, C, G or T (exact per byte: no
// borrow crosses bytes), and the 2-bit codes of 8 bases packed into 2 code bytes
inline uint64_t zero_bytes(uint64_t x) {
    const uint64_t m = 0x7F7F7F7F7F7F7F7Full;
    return ~(((x & m) + m) | x | m);
}
inline uint64_t exc_mask8(uint64_t w) {
    const uint64_t one = 0x0101010101010101ull;
    const uint64_t ok = zero_bytes(w ^ ('A' * one)) | zero_bytes(w ^ ('C' * one)) | zero_bytes(w ^ ('G' * one)) |
                        zero_bytes(w ^ ('T' * one));
    return ~ok & 0x8080808080808080ull;
}
inline uint16_t pack8(uint64_t w) {  // base j's code at bits 2 (j mod 4) of code byte j / 4
    const uint64_t c = ((w >> 1) ^ (w >> 2)) & 0x0303030303030303ull;
    const uint64_t x = c | (c >> 6) | (c >> 12) | (c >> 18);
    return (uint16_t)((x & 0xFF) | ((x >> 24) & 0xFF00));
}
inline uint64_t load8(const uint8_t *p) {
    uint64_t w;
    memcpy(&w, p, 8);
    return w;
}
#if defined(__SSE2__) && !defined(__HIP_DEVICE_COMPILE__)  // (host pass only)
// 16 bytes at a time (SSE2 is baseline x86-64): bit i set iff byte i is not A/C/G/T
inline unsigned exc_mask16(__m128i v) {
    const __m128i ok = _mm_or_si128(_mm_or_si128(_mm_cmpeq_epi8(v, _mm_set1_epi8('A')), _mm_cmpeq_epi8(v, _mm_set1_epi8('C'))),
                                    _mm_or_si128(_mm_cmpeq_epi8(v, _mm_set1_epi8('G')), _mm_cmpeq_epi8(v, _mm_set1_epi8('T'))));
    return ~(unsigned)_mm_movemask_epi8(ok) & 0xFFFFu;
}
// 16 bases -> 4 code bytes (base j at bits 2 (j mod 4) of byte j / 4)
inline uint32_t pack16(__m128i v) {
    const __m128i m3 = _mm_set1_epi8(3);
    const __m128i c = _mm_and_si128(_mm_xor_si128(_mm_srli_epi16(v, 1), _mm_srli_epi16(v, 2)), m3);
    __m128i x = _mm_or_si128(_mm_or_si128(c, _mm_srli_epi32(c, 6)), _mm_or_si128(_mm_srli_epi32(c, 12), _mm_srli_epi32(c, 18)));
    x = _mm_and_si128(x, _mm_set1_epi32(0xFF));
    x = _mm_packs_epi32(x, x);
    x = _mm_packus_epi16(x, x);
    return (uint32_t)_mm_cvtsi128_si32(x);
}
#endif
inline uint64_t count_exc(const uint8_t *p, uint64_t n) {
    uint64_t e = 0, i = 0;
#if defined(__SSE2__) && !defined(__HIP_DEVICE_COMPILE__)  // (host pass only)
    for (; i + 16 <= n; i += 16) e += (uint64_t)__builtin_popcount(exc_mask16(_mm_loadu_si128((const __m128i *)(p + i))));
#endif
    for (; i + 8 <= n; i += 8) e += (uint64_t)__builtin_popcountll(exc_mask8(load8(p + i)));
    for (; i < n; i++) e += is_exc(p[i]);
    return e;
}
// the next '\n' at or after s (hi if none): inline, no call per short line
inline uint64_t find_nl(const uint8_t *p, uint64_t s, uint64_t hi) {
#if defined(__SSE2__) && !defined(__HIP_DEVICE_COMPILE__)  // (host pass only)
    const __m128i nl = _mm_set1_epi8('\n');
    for (; s + 16 <= hi; s += 16) {
        const unsigned m = (unsigned)_mm_movemask_epi8(_mm_cmpeq_epi8(_mm_loadu_si128((const __m128i *)(p + s)), nl));
        if (m) return s + (uint64_t)__builtin_ctz(m);
    }
#endif
    for (; s < hi; s++)
        if (p[s] == '\n') return s;
    return hi;
}

// page-locked code buffers are reused across loads (pinning ~250 MB costs tens of ms): one
// cached buffer, handed out when large enough and returned by ec_reads_free
std::mutex g_pool_mu;
uint8_t *g_pool_p = nullptr;
size_t g_pool_cap = 0;
uint8_t *pinned_take(size_t n, size_t *cap) {
    {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        if (g_pool_p && g_pool_cap >= n) {
            uint8_t *q = g_pool_p;
            *cap = g_pool_cap;
            g_pool_p = nullptr;
            g_pool_cap = 0;
            return q;
        }
    }
    uint8_t *q = nullptr;
    if (hipHostMalloc((void **)&q, n, hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    *cap = n;
    return q;
}
void pinned_give(uint8_t *q, size_t cap) {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    if (g_pool_p && g_pool_cap >= cap) {
        (void)hipHostFree(q);
        return;
    }
    if (g_pool_p) (void)hipHostFree(g_pool_p);
    g_pool_p = q;
    g_pool_cap = cap;
}

// visit the lines of [lo, hi): fn(line_begin, line_end_excl_newline)
template <typename Fn>
void for_lines(const uint8_t *p, uint64_t lo, uint64_t hi, Fn fn) {
    uint64_t s = lo;
    while (s < hi) {
        const uint64_t e = find_nl(p, s, hi);
        fn(s, e);
        s = e + 1;
    }
}

// worker threads: the caller's count, else OMP_NUM_THREADS / the hardware (a GPU box's share
// of a many-core host is what OMP_NUM_THREADS says)
int host_threads(int threads) {
    if (threads > 0) return threads;
    const char *e = getenv("OMP_NUM_THREADS");
    const int env = e ? atoi(e) : 0;
    const int hw = (int)std::max(1u, std::thread::hardware_concurrency());
    return std::max(1, std::min(env > 0 ? env : hw, 64));
}

}  // namespace

ec_reads::~ec_reads() {
    if (codes && pinned) {
        // a staged batch's copy (ec_stage_packed_host returns before it ends) must not read a
        // buffer the next load is already refilling: the copies of that device drain first
        if (staged_dev >= 0) {
            int cur = 0;
            (void)hipGetDevice(&cur);
            (void)hipSetDevice(staged_dev);
            (void)hipDeviceSynchronize();
            (void)hipSetDevice(cur);
        }
        pinned_give(codes, codes_cap);
    } else {
        free(codes);
    }
}

extern "C" {

int ec_reads_load(const char *path, int format, int threads, ec_reads **out) {
    const bool pack = (format & EC_READS_PACKED) != 0;
    format &= ~EC_READS_PACKED;
    if (!path || !out || format < EC_FASTA_RECORDS || format > EC_FASTQ) {
        set_error("bad arguments");
        return EC_ERR_ARG;
    }
    *out = nullptr;
    const bool tdbg = getenv("EULERHIP_INGEST_TIMING") != nullptr;
    auto now = [] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    const double t_start = now();
    const int fd = open(path, O_RDONLY);
    if (fd < 0) {
        set_error("cannot open %s", path);
        return EC_ERR_ARG;
    }
    struct stat stt;
    if (fstat(fd, &stt) != 0) {
        close(fd);
        set_error("cannot stat %s", path);
        return EC_ERR_ARG;
    }
    const uint64_t n = (uint64_t)stt.st_size;
    const uint8_t *p = nullptr;
    if (n) {
        void *m = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
        if (m == MAP_FAILED) {
            close(fd);
            set_error("mmap of %s failed", path);
            return EC_ERR_NOMEM;
        }
        madvise(m, n, MADV_SEQUENTIAL);
        p = static_cast<const uint8_t *>(m);
    }
    close(fd);
    ec_reads *r = new (std::nothrow) ec_reads();
    if (!r) {
        if (p) munmap((void *)p, n);
        set_error("out of host memory");
        return EC_ERR_NOMEM;
    }
    int T = host_threads(threads);
    if (n < (1u << 20)) T = 1;
    // chunk boundaries at line starts
    std::vector<Chunk> ch(T);
    for (int t = 0; t < T; t++) {
        uint64_t lo = n * (uint64_t)t / T;
        if (t) {
            while (lo < n && p[lo - 1] != '\n') lo++;
        }
        ch[t].lo = lo;
    }
    for (int t = 0; t < T; t++) ch[t].hi = t + 1 < T ? ch[t + 1].lo : n;

    // pass 1: counts (and FASTQ line counts)
    auto pass1 = [&](int t) {
        Chunk &c = ch[t];
        if (format == EC_FASTQ) {
            uint64_t lines = 0;
            for_lines(p, c.lo, c.hi, [&](uint64_t, uint64_t) { lines++; });
            c.reads = lines;  // temporarily: line count
        } else if (format == EC_FASTA_LINES) {
            for_lines(p, c.lo, c.hi, [&](uint64_t b, uint64_t e) {
                if (b < e && p[b] == '>') return;
                strip(p, b, e);
                c.reads++;
                c.bases += e - b;
                if (pack) c.exc += count_exc(p + b, e - b);
            });
        } else {
            for_lines(p, c.lo, c.hi, [&](uint64_t b, uint64_t e) {
                if (b < e && p[b] == '>') {
                    c.reads++;
                    return;
                }
                strip(p, b, e);
                c.bases += e - b;  // bases before the chunk's first header are resolved below
                if (pack) c.exc += count_exc(p + b, e - b);
            });
        }
    };
    {
        std::vector<std::thread> th;
        for (int t = 1; t < T; t++) th.emplace_back(pass1, t);
        pass1(0);
        for (auto &x : th) x.join();
    }
    if (format == EC_FASTQ) {
        uint64_t lines = 0;
        for (auto &c : ch) {
            c.lines_before = lines;
            lines += c.reads;
        }
        // file ends without a trailing newline-only line: a partial last record still counts
        // its sequence line (read_fastq yields every line with index % 4 == 1)
        for (auto &c : ch) {
            c.reads = 0;
            c.bases = 0;
        }
        auto pass1b = [&](int t) {
            Chunk &c = ch[t];
            uint64_t li = c.lines_before;
            for_lines(p, c.lo, c.hi, [&](uint64_t b, uint64_t e) {
                if (li % 4 == 1) {
                    if (e > b && p[e - 1] == '\r') e--;  // rstrip('\n') of a CRLF line keeps '\r'; drop it
                    c.reads++;
                    c.bases += e - b;
                    if (pack) c.exc += count_exc(p + b, e - b);
                }
                li++;
            });
        };
        std::vector<std::thread> th;
        for (int t = 1; t < T; t++) th.emplace_back(pass1b, t);
        pass1b(0);
        for (auto &x : th) x.join();
    }
    const double t_p1 = now();
    // FASTA records: sequence bytes before a chunk's first header belong to the previous
    // chunk's last record (or to no record at the file start)
    std::vector<uint64_t> lead(T, 0), lead_exc(T, 0);
    if (format == EC_FASTA_RECORDS) {
        auto lead_of = [&](int t) {  // stripped bytes before the chunk's first header
            uint64_t sum = 0, q = ch[t].lo, ex = 0;
            while (q < ch[t].hi) {
                const void *nl = memchr(p + q, '\n', ch[t].hi - q);
                uint64_t e = nl ? (uint64_t)((const uint8_t *)nl - p) : ch[t].hi;
                if (q < e && p[q] == '>') break;
                uint64_t b = q;
                const uint64_t next = e + 1;
                strip(p, b, e);
                sum += e - b;
                if (pack) ex += count_exc(p + b, e - b);
                q = next;
            }
            lead[t] = sum;
            lead_exc[t] = ex;
        };
        for (int t = 0; t < T; t++) lead_of(t);
        // chunk t's leading bytes: counted by chunk t, belong to the last record before it
        bool any_header_before = false;
        for (int t = 0; t < T; t++) {
            if (!any_header_before) ch[t].bases -= lead[t], ch[t].exc -= lead_exc[t];  // no record yet: ignored text
            any_header_before |= ch[t].reads > 0;
        }
    }
    uint64_t R = 0, B = 0, X = 0;
    std::vector<uint64_t> r0(T), b0(T), x0(T);
    for (int t = 0; t < T; t++) {
        r0[t] = R;
        b0[t] = B;
        x0[t] = X;
        R += ch[t].reads;
        B += ch[t].bases;
        X += ch[t].exc;
    }
    try {
        if (pack) {
            r->packed = true;
            r->nbases = B;
            const uint64_t nc = (B + 3) / 4 + 16;
            // page-locked so the codes go over PCIe at DMA speed; a host without a usable GPU
            // (ingest tests on CPU) gets ordinary memory
            r->codes = pinned_take(nc, &r->codes_cap);
            if (!r->codes) {
                r->codes = static_cast<uint8_t *>(malloc(nc));
                if (!r->codes) throw std::bad_alloc();
                r->pinned = false;
            }
            // (zeroed by the copy threads: each its own code bytes, pass 2 below)
            r->exc_pos.resize(X);
            r->exc_byte.resize(X);
        } else {
            r->bases.resize(std::max<uint64_t>(B, 1));
        }
        r->offsets.resize(R + 1);
    } catch (...) {
        delete r;
        if (p) munmap((void *)p, n);
        set_error("out of host memory (%llu reads, %llu bases)", (unsigned long long)R, (unsigned long long)B);
        return EC_ERR_NOMEM;
    }
    uint8_t *ob = r->bases.data();
    uint64_t *oo = r->offsets.data();
    uint8_t *oc = r->codes;
    uint64_t *xp = r->exc_pos.data();
    uint8_t *xb = r->exc_byte.data();
    // pass 2: copy.  Record reads get offsets[i] at their header; their bytes follow contiguously
    // across chunk boundaries because b0 is a prefix sum in file order.
    auto pass2 = [&](int t) {
        const Chunk &c = ch[t];
        uint64_t ri = r0[t], bi = b0[t], xi = x0[t];
        // packed: the code bytes of bases [b0[t], b0[t + 1]) -- the first and the last may be
        // shared with the neighbouring chunks' bases (atomic OR there; the last chunk shares
        // none at its end).  Whole code bytes (4 bases of this chunk) are plain stores.
        const uint64_t cb0 = b0[t] >> 2, cbl = t + 1 < T ? b0[t + 1] >> 2 : ~0ull;
        auto put1 = [&](uint8_t ch8) {
            const uint8_t v = (uint8_t)(code2(ch8) << (2 * (bi & 3)));
            const uint64_t cb = bi >> 2;
            if (cb == cb0 || cb == cbl) __atomic_fetch_or(oc + cb, v, __ATOMIC_RELAXED);
            else oc[cb] |= v;
            if (is_exc(ch8)) xp[xi] = bi, xb[xi++] = ch8;
            bi++;
        };
        auto put = [&](const uint8_t *src, uint64_t n) {
            if (!pack) {
                memcpy(ob + bi, src, n);
                bi += n;
                return;
            }
            uint64_t i = 0;
            for (; i < n && (bi & 3); i++) put1(src[i]);
#if defined(__SSE2__) && !defined(__HIP_DEVICE_COMPILE__)  // (host pass only)
            for (; i + 16 <= n; i += 16) {  // 16 bases -> 4 whole code bytes
                const __m128i v = _mm_loadu_si128((const __m128i *)(src + i));
                const uint32_t c = pack16(v);
                memcpy(oc + (bi >> 2), &c, 4);
                unsigned bad = exc_mask16(v);
                while (bad) {
                    const int j = __builtin_ctz(bad);
                    xp[xi] = bi + j, xb[xi++] = src[i + j];
                    bad &= bad - 1;
                }
                bi += 16;
            }
#endif
            for (; i + 8 <= n; i += 8) {  // 8 bases -> 2 whole code bytes
                const uint64_t w = load8(src + i);
                const uint16_t c = pack8(w);
                memcpy(oc + (bi >> 2), &c, 2);
                uint64_t bad = exc_mask8(w);
                while (bad) {
                    const int j = __builtin_ctzll(bad) >> 3;
                    xp[xi] = bi + j, xb[xi++] = src[i + j];
                    bad &= bad - 1;
                }
                bi += 8;
            }
            for (; i < n; i++) put1(src[i]);
        };
        if (pack) {  // zero this chunk's code bytes (whole ones; the shared boundary bytes were zeroed before)
            const uint64_t z0 = (b0[t] + 3) >> 2, z1 = t + 1 < T ? b0[t + 1] >> 2 : (B + 3) / 4 + 16;
            if (z1 > z0) memset(oc + z0, 0, z1 - z0);
        }
        if (format == EC_FASTQ) {
            uint64_t li = c.lines_before;
            for_lines(p, c.lo, c.hi, [&](uint64_t b, uint64_t e) {
                if (li % 4 == 1) {
                    if (e > b && p[e - 1] == '\r') e--;
                    oo[ri++] = bi;
                    put(p + b, e - b);
                }
                li++;
            });
        } else if (format == EC_FASTA_LINES) {
            for_lines(p, c.lo, c.hi, [&](uint64_t b, uint64_t e) {
                if (b < e && p[b] == '>') return;
                strip(p, b, e);
                oo[ri++] = bi;
                put(p + b, e - b);
            });
        } else {
            const bool owned_lead = ri > 0;  // leading bytes continue the previous record
            bool in_lead = true;
            for_lines(p, c.lo, c.hi, [&](uint64_t b, uint64_t e) {
                if (b < e && p[b] == '>') {
                    in_lead = false;
                    oo[ri++] = bi;
                    return;
                }
                if (in_lead && !owned_lead) return;
                strip(p, b, e);
                put(p + b, e - b);
            });
        }
    };
    const double t_alloc = now();
    if (pack)  // code bytes shared by two chunks' bases: zeroed before the chunks OR into them
        for (int t = 0; t < T; t++)
            if (b0[t] & 3) oc[b0[t] >> 2] = 0;
    {
        std::vector<std::thread> th;
        for (int t = 1; t < T; t++) th.emplace_back(pass2, t);
        pass2(0);
        for (auto &x : th) x.join();
    }
    oo[R] = B;
    const double t_p2 = now();
    if (p) munmap((void *)p, n);
    if (tdbg)
        fprintf(stderr, "ingest: T %d pass1 %.1f alloc %.1f pass2 %.1f munmap %.1f ms\n", T, t_p1 - t_start,
                t_alloc - t_p1, t_p2 - t_alloc, now() - t_p2);
    if (pack && R) {  // one read length: no offsets travel
        const uint64_t L = oo[1] - oo[0];
        bool one = L <= 0xFFFFFFFFull;
        for (uint64_t i = 0; i < R && one; i++) one = oo[i + 1] - oo[i] == L;
        r->read_len = one ? (uint32_t)L : 0u;
    }
    *out = r;
    return EC_OK;
}

int ec_reads_packed_info(const ec_reads *r, uint64_t *nbases, uint32_t *read_len, uint64_t *n_exc) {
    if (!r || !r->packed) {
        set_error("not a packed read set (ec_reads_load with EC_READS_PACKED)");
        return EC_ERR_ARG;
    }
    if (nbases) *nbases = r->nbases;
    if (read_len) *read_len = r->read_len;
    if (n_exc) *n_exc = r->exc_pos.size();
    return EC_OK;
}

int ec_reads_packed_copy(const ec_reads *r, uint8_t *codes, uint64_t *exc_pos, uint8_t *exc_byte) {
    if (!r || !r->packed) {
        set_error("not a packed read set (ec_reads_load with EC_READS_PACKED)");
        return EC_ERR_ARG;
    }
    if (codes && r->nbases) memcpy(codes, r->codes, (r->nbases + 3) / 4);
    if (exc_pos && !r->exc_pos.empty()) memcpy(exc_pos, r->exc_pos.data(), r->exc_pos.size() * 8);
    if (exc_byte && !r->exc_byte.empty()) memcpy(exc_byte, r->exc_byte.data(), r->exc_byte.size());
    return EC_OK;
}

// a packed read set as a staged batch (ec_stage_packed_host)
int ec_stage_packed_reads(ec_session *s, const ec_reads *r) {
    if (!r || !r->packed) {
        set_error("not a packed read set (ec_reads_load with EC_READS_PACKED)");
        return EC_ERR_ARG;
    }
    const uint64_t R = r->offsets.size() - 1;
    const int rc = ec_stage_packed_host(s, r->codes, r->nbases, r->read_len ? nullptr : r->offsets.data(), R,
                                        r->read_len, r->exc_pos.empty() ? nullptr : r->exc_pos.data(),
                                        r->exc_byte.empty() ? nullptr : r->exc_byte.data(), r->exc_pos.size());
    int dev = 0;  // (ec_stage_packed_host made the session's device current)
    if (hipGetDevice(&dev) == hipSuccess) const_cast<ec_reads *>(r)->staged_dev = dev;
    return rc;
}

// the fused assembly straight from a packed read set (its page-locked codes go over PCIe)
int ec_assemble_packed_reads(ec_session *s, const ec_reads *r, int k, int limit, unsigned flags) {
    if (!r || !r->packed) {
        set_error("not a packed read set (ec_reads_load with EC_READS_PACKED)");
        return EC_ERR_ARG;
    }
    const uint64_t R = r->offsets.size() - 1;
    return ec_assemble_packed_host(s, r->codes, r->nbases, r->read_len ? nullptr : r->offsets.data(), R, r->read_len,
                                   r->exc_pos.empty() ? nullptr : r->exc_pos.data(),
                                   r->exc_byte.empty() ? nullptr : r->exc_byte.data(), r->exc_pos.size(), k, limit,
                                   flags);
}

uint64_t ec_reads_count(const ec_reads *r) { return r ? r->offsets.size() - 1 : 0; }

uint64_t ec_reads_bases(const ec_reads *r) { return r ? r->offsets.back() : 0; }

uint64_t ec_reads_span(const ec_reads *r, uint64_t first, uint64_t count) {
    if (!r || first + count > r->offsets.size() - 1) return 0;
    return r->offsets[first + count] - r->offsets[first];
}

int ec_reads_copy(const ec_reads *r, uint64_t first, uint64_t count, uint8_t *bases, uint64_t *offsets) {
    if (r && r->packed && bases && count) {
        set_error("a packed read set holds no ASCII bases (ec_reads_packed_copy)");
        return EC_ERR_ARG;
    }
    if (!r || first + count > r->offsets.size() - 1 || (count && !offsets)) {
        set_error("bad shard [%llu, +%llu)", (unsigned long long)first, (unsigned long long)count);
        return EC_ERR_ARG;
    }
    const uint64_t b0 = r->offsets[first], b1 = r->offsets[first + count];
    if (b1 > b0 && !bases && !r->packed) {
        set_error("null base buffer");
        return EC_ERR_ARG;
    }
    if (b1 > b0 && bases) memcpy(bases, r->bases.data() + b0, b1 - b0);
    for (uint64_t i = 0; i <= count; i++) offsets[i] = r->offsets[first + i] - b0;
    return EC_OK;
}

void ec_reads_free(ec_reads *r) { delete r; }

void ec_reads_release_pool(void) {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    if (g_pool_p) (void)hipHostFree(g_pool_p);
    g_pool_p = nullptr;
    g_pool_cap = 0;
}

// ASCII -> 2 bits per base + exceptions (ec_assemble_packed_host's layout).  Threads own
// base ranges aligned to 4 (whole code bytes); exceptions are counted per range, then written
// at prefix-summed positions so they stay ascending.
int ec_pack_reads(const uint8_t *reads, const uint64_t *offsets, uint64_t nreads, int threads, uint8_t *codes,
                  uint64_t *exc_pos, uint8_t *exc_byte, uint64_t exc_cap, uint64_t *n_exc, uint32_t *read_len) {
    if (!offsets || !n_exc || !read_len) {
        set_error("null argument");
        return EC_ERR_ARG;
    }
    if (nreads == UINT64_MAX) {  // (nreads + 1 offsets: an empty offsets array passed as -1)
        set_error("bad read count");
        return EC_ERR_ARG;
    }
    if (offsets[0] != 0) {
        set_error("offsets[0] = %llu, not 0", (unsigned long long)offsets[0]);
        return EC_ERR_ARG;
    }
    for (uint64_t r = 0; r < nreads; r++)
        if (offsets[r + 1] < offsets[r]) {
            set_error("offsets not monotone at read %llu", (unsigned long long)r);
            return EC_ERR_ARG;
        }
    const uint64_t nb = offsets[nreads];
    if (nb && (!reads || !codes)) {
        set_error("null reads / codes");
        return EC_ERR_ARG;
    }
    int T = host_threads(threads);
    if (nb < (1u << 22)) T = 1;
    std::vector<uint64_t> lo(T + 1), nexc(T, 0);
    for (int t = 0; t <= T; t++) lo[t] = t == T ? nb : (nb * (uint64_t)t / T) & ~3ull;
    std::vector<uint8_t> uni(T, 1);
    // code of an ASCII byte (A 0, C 1, G 2, T 3) and whether the byte is exactly that letter
    auto code = [](uint8_t c) { return (uint8_t)(((c >> 1) ^ (c >> 2)) & 3u); };
    static const uint8_t letter[4] = {'A', 'C', 'G', 'T'};
    auto pass = [&](int t, bool write) {
        uint64_t e = 0, ebase = 0;
        if (write)
            for (int q = 0; q < t; q++) ebase += nexc[q];
        for (uint64_t i = lo[t]; i < lo[t + 1]; i += 4) {
            uint8_t byte = 0;
            const int n = (int)std::min<uint64_t>(4, lo[t + 1] - i);
            for (int j = 0; j < n; j++) {
                const uint8_t c = reads[i + j], x = code(c);
                byte |= (uint8_t)(x << (2 * j));
                if (letter[x] != c) {
                    if (write && ebase + e < exc_cap) {
                        exc_pos[ebase + e] = i + j;
                        exc_byte[ebase + e] = c;
                    }
                    e++;
                }
            }
            if (write) codes[i >> 2] = byte;
        }
        if (!write) nexc[t] = e;
        // one read length?  (reads [t n / T, (t + 1) n / T))
        if (!write && nreads) {
            const uint64_t r0 = nreads * (uint64_t)t / T, r1 = nreads * (uint64_t)(t + 1) / T;
            const uint64_t L = offsets[1] - offsets[0];
            for (uint64_t r = r0; r < r1; r++)
                if (offsets[r + 1] - offsets[r] != L) {
                    uni[t] = 0;
                    break;
                }
        }
    };
    for (int phase = 0; phase < 2; phase++) {  // count, then write
        std::vector<std::thread> th;
        for (int t = 1; t < T; t++) th.emplace_back(pass, t, phase == 1);
        pass(0, phase == 1);
        for (auto &x : th) x.join();
    }
    uint64_t tot = 0;
    for (auto v : nexc) tot += v;
    *n_exc = tot;
    bool one = true;
    for (auto v : uni) one &= v != 0;
    const uint64_t L = nreads ? offsets[1] - offsets[0] : 0;
    *read_len = (one && nreads && L <= 0xFFFFFFFFull && offsets[0] == 0) ? (uint32_t)L : 0u;
    return EC_OK;
}

}  // extern "C"
