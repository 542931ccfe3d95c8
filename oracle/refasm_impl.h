/* oracle/refasm_impl.h -- TEST INFRASTRUCTURE ONLY.  Included twice by refasm.c with
 * KEY = uint64_t / unsigned __int128 and SFX = _64 / _128.  Every function restates one
 * function of src/referenceassembler/referenceAssembler.py (line cited). */
#define CAT2(a, b) a##b
#define CAT(a, b) CAT2(a, b)
#define F(name) CAT(name, SFX)

/* ---- insertion-ordered map KEY -> u32 (stands in for the Python dict, build:26) ---- */
typedef struct {
    KEY *keys;
    uint32_t *vals;
    uint64_t n, ncap;
    uint32_t *slots; /* entry index + 1, 0 = empty */
    uint64_t smask;
} F(omap);

static int F(om_init)(F(omap) *m, uint64_t cap) {
    uint64_t s = 1024;
    while (s < 2 * cap) s <<= 1;
    memset(m, 0, sizeof(*m));
    m->ncap = cap < 16 ? 16 : cap;
    m->keys = (KEY *)malloc(m->ncap * sizeof(KEY));
    m->vals = (uint32_t *)malloc(m->ncap * sizeof(uint32_t));
    m->slots = (uint32_t *)calloc(s, sizeof(uint32_t));
    m->smask = s - 1;
    return (m->keys && m->vals && m->slots) ? 0 : -3;
}

static void F(om_free)(F(omap) *m) { free(m->keys); free(m->vals); free(m->slots); }

static int64_t F(om_find)(const F(omap) *m, KEY key) {
    uint64_t h = KHASH(key) & m->smask;
    for (;;) {
        uint32_t s = m->slots[h];
        if (!s) return -1;
        if (m->keys[s - 1] == key) return (int64_t)(s - 1);
        h = (h + 1) & m->smask;
    }
}

static int F(om_rehash)(F(omap) *m, uint64_t nslots) {
    free(m->slots);
    m->slots = (uint32_t *)calloc(nslots, sizeof(uint32_t));
    if (!m->slots) return -3;
    m->smask = nslots - 1;
    for (uint64_t i = 0; i < m->n; i++) {
        uint64_t h = KHASH(m->keys[i]) & m->smask;
        while (m->slots[h]) h = (h + 1) & m->smask;
        m->slots[h] = (uint32_t)(i + 1);
    }
    return 0;
}

/* d[key] += add, inserting at the end if absent (defaultdict(int) semantics, build:26,32,35) */
static int F(om_add)(F(omap) *m, KEY key, uint32_t add) {
    uint64_t h = KHASH(key) & m->smask;
    for (;;) {
        uint32_t s = m->slots[h];
        if (!s) break;
        if (m->keys[s - 1] == key) { m->vals[s - 1] += add; return 0; }
        h = (h + 1) & m->smask;
    }
    if (m->n == m->ncap) {
        m->ncap *= 2;
        KEY *nk = (KEY *)realloc(m->keys, m->ncap * sizeof(KEY));
        uint32_t *nv = (uint32_t *)realloc(m->vals, m->ncap * sizeof(uint32_t));
        if (!nk || !nv) return -3;
        m->keys = nk; m->vals = nv;
    }
    m->keys[m->n] = key;
    m->vals[m->n] = add;
    m->n++;
    m->slots[h] = (uint32_t)m->n;
    if (2 * m->n > m->smask) return F(om_rehash)(m, 2 * (m->smask + 1));
    return 0;
}

/* set semantics with overwrite (heads/tails dicts of all_contigs:91-96) */
static int F(om_set)(F(omap) *m, KEY key, uint32_t v) {
    int64_t e = F(om_find)(m, key);
    if (e >= 0) { m->vals[e] = v; return 0; }
    return F(om_add)(m, key, v);
}

/* ---- 2-bit string algebra ----------------------------------------------------------- */
static inline KEY F(kmask)(int k) {
    return (2 * k >= (int)(8 * sizeof(KEY))) ? (KEY)~(KEY)0 : (((KEY)1 << (2 * k)) - 1);
}

static inline uint64_t F(rev2_64)(uint64_t x) {
    x = ((x >> 2) & 0x3333333333333333ULL) | ((x & 0x3333333333333333ULL) << 2);
    x = ((x >> 4) & 0x0F0F0F0F0F0F0F0FULL) | ((x & 0x0F0F0F0F0F0F0F0FULL) << 4);
    return __builtin_bswap64(x);
}

/* twin(km) = reverse complement (referenceAssembler.py:7-10) */
static inline KEY F(twin)(KEY x, int k) {
    KEY c = x ^ F(kmask)(k);
    if (sizeof(KEY) == 8) return (KEY)(F(rev2_64)((uint64_t)c) >> (64 - 2 * k));
    u128 lo = (u128)F(rev2_64)((uint64_t)c), hi = (u128)F(rev2_64)((uint64_t)((u128)c >> 64));
    u128 r = (lo << 64) | hi;
    return (KEY)(r >> (128 - 2 * k));
}

/* fw:16-18 -> km[1:]+x ; bw:20-22 -> x+km[:-1] (x in 'ACGT' order = codes 0..3) */
static inline KEY F(fwn)(KEY x, int b, int k) { return ((x << 2) | (KEY)b) & F(kmask)(k); }
static inline KEY F(bwn)(KEY x, int b, int k) { return ((KEY)b << (2 * (k - 1))) | (x >> 2); }

static inline int F(in_d)(const F(omap) *d, KEY x) { return F(om_find)(d, x) >= 0; }

/* ---- build:25-42 -------------------------------------------------------------------- */
static int F(insert_seq)(F(omap) *d, const unsigned char *s, uint64_t len, int k, int twin_strand) {
    /* for km in kmers(seq,k): d[km] += 1 (build:31-32 forward, :33-35 on twin(seg)) */
    const KEY mask = F(kmask)(k);
    KEY code = 0;
    static const int comp[4] = {3, 2, 1, 0};
    for (uint64_t t = 0; t < len; t++) {
        int b = twin_strand ? comp[base_code(s[len - 1 - t])] : base_code(s[t]);
        code = ((code << 2) | (KEY)b) & mask;
        if (t + 1 >= (uint64_t)k) {
            int rc = F(om_add)(d, code, 1);
            if (rc) return rc;
        }
    }
    return 0;
}

/* ---- get_contig_forward:59-77 --------------------------------------------------------- */
typedef struct { KEY *v; uint64_t n, cap; } F(kvec);
static int F(kv_push)(F(kvec) *a, KEY x) {
    if (a->n == a->cap) {
        a->cap = a->cap ? 2 * a->cap : 64;
        KEY *nv = (KEY *)realloc(a->v, a->cap * sizeof(KEY));
        if (!nv) return -3;
        a->v = nv;
    }
    a->v[a->n++] = x;
    return 0;
}

static int F(contig_forward)(const F(omap) *d, KEY km, int k, F(kvec) *c) {
    c->n = 0;
    if (F(kv_push)(c, km)) return -3;
    const KEY tkm = F(twin)(km, k);
    for (;;) {
        KEY last = c->v[c->n - 1], cand = 0;
        int n = 0;
        for (int b = 0; b < 4; b++) {
            KEY y = F(fwn)(last, b, k);
            if (F(in_d)(d, y)) { if (!n) cand = y; n++; }
        }
        if (n != 1) break;
        if (cand == km || cand == tkm) break;        /* cycles / Moebius (:67-68) */
        if (cand == F(twin)(last, k)) break;          /* hairpins (:69-70) */
        int nb = 0;
        for (int b = 0; b < 4; b++) nb += F(in_d)(d, F(bwn)(cand, b, k));
        if (nb != 1) break;                           /* :72-73 */
        if (F(kv_push)(c, cand)) return -3;
    }
    return 0;
}

/* ---- string output helpers ------------------------------------------------------------ */
typedef struct { char *p; uint64_t n, cap; } F(cbuf);
static int F(cb_reserve)(F(cbuf) *b, uint64_t extra) {
    if (b->n + extra <= b->cap) return 0;
    uint64_t nc = b->cap ? b->cap : 1024;
    while (nc < b->n + extra) nc *= 2;
    char *np = (char *)realloc(b->p, nc);
    if (!np) return -3;
    b->p = np; b->cap = nc;
    return 0;
}
static void F(put_kmer)(char *dst, KEY x, int k) {
    static const char A[4] = {'A', 'C', 'G', 'T'};
    for (int i = k - 1; i >= 0; i--) { dst[i] = A[(int)(x & 3)]; x >>= 2; }
}

/* one read's N-split segments (build:29): calls seg(s + p, q - p) for every segment of >= k
 * bases; -2 on a byte outside {A,C,G,T,N} */
#define SEGMENTS(r, s, len, k, SEG_BODY)                                                              \
    do {                                                                                              \
        uint64_t p_ = 0;                                                                              \
        while (p_ <= (len)) {                                                                         \
            uint64_t q_ = p_;                                                                         \
            while (q_ < (len) && (s)[q_] != 'N') {                                                    \
                if (base_code((s)[q_]) < 0) {                                                         \
                    snprintf(g_err, sizeof g_err, "read %llu byte %llu (0x%02x) outside {A,C,G,T,N}", \
                             (unsigned long long)(r), (unsigned long long)q_, (s)[q_]);               \
                    rc = -2;                                                                          \
                    goto fail;                                                                        \
                }                                                                                     \
                q_++;                                                                                 \
            }                                                                                         \
            if (q_ - p_ >= (uint64_t)(k)) {                                                           \
                const unsigned char *seg = (s) + p_;                                                  \
                const uint64_t seglen = q_ - p_;                                                      \
                SEG_BODY;                                                                             \
            }                                                                                         \
            p_ = q_ + 1;                                                                              \
        }                                                                                             \
    } while (0)

/* build:25-42 -> d (insertion-ordered, entries with count > limit) */
static int F(build)(const char *buf, const uint64_t *offsets, uint64_t nreads, int k, int limit, F(omap) *d,
                    uint64_t *npos) {
    int rc = 0;
    if ((rc = F(om_init)(d, 1 << 16))) return rc;
    /* build:27-35 -- per read, per N-split segment, forward then twin(seg) k-mers */
    for (uint64_t r = 0; r < nreads; r++) {
        const unsigned char *s = (const unsigned char *)buf + offsets[r];
        uint64_t len = offsets[r + 1] - offsets[r];
        SEGMENTS(r, s, len, k, {
            *npos += seglen - k + 1;
            if ((rc = F(insert_seq)(d, seg, seglen, k, 0))) goto fail;
            if ((rc = F(insert_seq)(d, seg, seglen, k, 1))) goto fail;
        });
    }
    /* build:37-39 -- delete d[x] <= limit, keeping insertion order */
    {
        uint64_t w = 0;
        for (uint64_t i = 0; i < d->n; i++)
            if ((int64_t)d->vals[i] > (int64_t)limit) { d->keys[w] = d->keys[i]; d->vals[w] = d->vals[i]; w++; }
        d->n = w;
        uint64_t s = 1024;
        while (s < 2 * (d->n + 1)) s <<= 1;
        if ((rc = F(om_rehash)(d, s))) goto fail;
    }
    return 0;
fail:
    return rc;
}

/* all_contigs:79-111 on d (consumed: freed on return) */
static int F(all_contigs)(F(omap) *dp, int k, unsigned flags, oracle_result *out);

static int F(assemble)(const char *buf, const uint64_t *offsets, uint64_t nreads, int k, int limit,
                       unsigned flags, oracle_result *out) {
    F(omap) d;
    memset(&d, 0, sizeof d);
    int rc = F(build)(buf, offsets, nreads, k, limit, &d, &out->n_positions);
    if (rc) {
        F(om_free)(&d);
        if (rc == -3) snprintf(g_err, sizeof g_err, "out of memory");
        return rc;
    }
    return F(all_contigs)(&d, k, flags, out);
}

static int F(all_contigs)(F(omap) *dp, int k, unsigned flags, oracle_result *out) {
    int rc = 0;
    F(omap) d = *dp, heads, tails;
    F(kvec) cf = {0}, cb = {0}, c = {0};
    F(cbuf) chars = {0};
    uint64_t *coff = NULL, *loff = NULL;
    int64_t *links = NULL;
    uint64_t nlinks = 0, lcap = 0, ncontig = 0, ccap = 0;
    unsigned char *done = NULL;
    memset(&heads, 0, sizeof heads);
    memset(&tails, 0, sizeof tails);
    out->n_dict = d.n;
    if (flags & ORACLE_WANT_DICT) {
        out->dict_kmers = (char *)malloc(d.n * (uint64_t)k + 1);
        out->dict_counts = (uint32_t *)malloc((d.n + 1) * sizeof(uint32_t));
        if (!out->dict_kmers || !out->dict_counts) { rc = -3; goto fail; }
        for (uint64_t i = 0; i < d.n; i++) {
            F(put_kmer)(out->dict_kmers + i * (uint64_t)k, d.keys[i], k);
            out->dict_counts[i] = d.vals[i];
        }
    }

    /* all_contigs:80-88 */
    done = (unsigned char *)calloc(d.n + 1, 1);
    coff = (uint64_t *)malloc(sizeof(uint64_t) * 1024);
    ccap = 1023;
    if (!done || !coff) { rc = -3; goto fail; }
    coff[0] = 0;
    for (uint64_t e = 0; e < d.n; e++) {
        if (done[e]) continue;
        KEY km = d.keys[e];
        /* get_contig:47-56 */
        if ((rc = F(contig_forward)(&d, km, k, &cf))) goto fail;
        if ((rc = F(contig_forward)(&d, F(twin)(km, k), k, &cb))) goto fail;
        c.n = 0;
        int cyc = 0;
        for (int b = 0; b < 4; b++) cyc |= (F(fwn)(cf.v[cf.n - 1], b, k) == km);
        if (!cyc)
            for (uint64_t i = cb.n - 1; i >= 1; i--)
                if ((rc = F(kv_push)(&c, F(twin)(cb.v[i], k)))) goto fail;
        for (uint64_t i = 0; i < cf.n; i++)
            if ((rc = F(kv_push)(&c, cf.v[i]))) goto fail;
        /* contig_to_string:44-45 */
        if ((rc = F(cb_reserve)(&chars, (uint64_t)k + c.n))) goto fail;
        F(put_kmer)(chars.p + chars.n, c.v[0], k);
        chars.n += k;
        for (uint64_t i = 1; i < c.n; i++) chars.p[chars.n++] = "ACGT"[(int)(c.v[i] & 3)];
        for (uint64_t i = 0; i < c.n; i++) {
            done[F(om_find)(&d, c.v[i])] = 1;
            int64_t t = F(om_find)(&d, F(twin)(c.v[i], k));
            if (t >= 0) done[t] = 1;
        }
        if (ncontig + 1 >= ccap) {
            ccap = 2 * ccap + 1;
            uint64_t *nc = (uint64_t *)realloc(coff, (ccap + 1) * sizeof(uint64_t));
            if (!nc) { rc = -3; goto fail; }
            coff = nc;
        }
        coff[++ncontig] = chars.n;
    }

    /* all_contigs:90-109 -- GFA links */
    if ((rc = F(om_init)(&heads, ncontig + 1)) || (rc = F(om_init)(&tails, ncontig + 1))) goto fail;
    for (uint64_t i = 0; i < ncontig; i++) {
        const unsigned char *x = (const unsigned char *)chars.p + coff[i];
        uint64_t L = coff[i + 1] - coff[i];
        KEY h = 0, t = 0;
        for (int j = 0; j < k; j++) h = (h << 2) | (KEY)base_code(x[j]);
        for (int j = 0; j < k; j++) t = (t << 2) | (KEY)base_code(x[L - k + j]);
        if ((rc = F(om_set)(&heads, h, (uint32_t)i))) goto fail;
        if ((rc = F(om_set)(&tails, F(twin)(t, k), (uint32_t)i))) goto fail;
    }
    loff = (uint64_t *)malloc((2 * ncontig + 1) * sizeof(uint64_t));
    if (!loff) { rc = -3; goto fail; }
    loff[0] = 0;
    for (uint64_t i = 0; i < ncontig; i++) {
        const unsigned char *x = (const unsigned char *)chars.p + coff[i];
        uint64_t L = coff[i + 1] - coff[i];
        KEY h = 0, t = 0;
        for (int j = 0; j < k; j++) h = (h << 2) | (KEY)base_code(x[j]);
        for (int j = 0; j < k; j++) t = (t << 2) | (KEY)base_code(x[L - k + j]);
        for (int side = 0; side < 2; side++) {
            KEY src = side == 0 ? t : F(twin)(h, k);
            for (int b = 0; b < 4; b++) {
                KEY y = F(fwn)(src, b, k);
                int64_t hh = F(om_find)(&heads, y), tt = F(om_find)(&tails, y);
                for (int which = 0; which < 2; which++) {
                    int64_t v = which == 0 ? hh : tt;
                    if (v < 0) continue;
                    if (nlinks == lcap) {
                        lcap = lcap ? 2 * lcap : 256;
                        int64_t *nl = (int64_t *)realloc(links, lcap * sizeof(int64_t));
                        if (!nl) { rc = -3; goto fail; }
                        links = nl;
                    }
                    links[nlinks++] = 2 * (int64_t)(which == 0 ? heads.vals[v] : tails.vals[v]) + which;
                }
            }
            loff[2 * i + side + 1] = nlinks;
        }
    }
    out->n_contigs = ncontig;
    out->contig_chars = chars.p;
    chars.p = NULL;
    out->contig_offsets = coff;
    coff = NULL;
    out->link_offsets = loff;
    loff = NULL;
    out->links = links;
    links = NULL;
fail:
    F(om_free)(&d);
    F(om_free)(&heads);
    F(om_free)(&tails);
    free(cf.v); free(cb.v); free(c.v); free(chars.p); free(coff); free(loff); free(links); free(done);
    if (rc == -3) snprintf(g_err, sizeof g_err, "out of memory");
    return rc;
}

/* ---- N-core variant (bench.py cpu_baseline "cores": N) ---------------------------------------
 * The reference's distributed CPU path, src/ref_spark.py:76-84: flatMap every read to its
 * forward and reverse-complement k-mers, map to (k-mer, 1), reduceByKey -- here T map threads
 * over contiguous read ranges, each combining into P = T hash partitions (Spark's map-side
 * combine), then P reduce threads merging one partition each.  Unlike ref_spark (whose
 * per-partition all_contigs loses the global dict), every entry also keeps the minimum
 * insertion event (read << 32 | index of the insert within the read, build:31-35), so sorting
 * the solid entries by event restores build()'s insertion order exactly; all_contigs then runs
 * single-threaded on that dict.  Results equal F(assemble)'s. */
typedef struct {
    KEY *keys;
    uint32_t *cnt;
    uint64_t *ev;
    uint64_t n, mask;
} F(cmap);

static int F(cm_init)(F(cmap) *m, uint64_t cap) {
    uint64_t s = 1024;
    while (s < 2 * cap) s <<= 1;
    m->keys = (KEY *)malloc(s * sizeof(KEY));
    m->cnt = (uint32_t *)calloc(s, sizeof(uint32_t));
    m->ev = (uint64_t *)malloc(s * sizeof(uint64_t));
    m->n = 0;
    m->mask = s - 1;
    return (m->keys && m->cnt && m->ev) ? 0 : -3;
}
static void F(cm_free)(F(cmap) *m) { free(m->keys); free(m->cnt); free(m->ev); memset(m, 0, sizeof *m); }

static int F(cm_add)(F(cmap) *m, KEY key, uint32_t add, uint64_t ev);
static int F(cm_grow)(F(cmap) *m) {
    F(cmap) o = *m;
    if (F(cm_init)(m, o.mask + 1)) return -3;
    for (uint64_t i = 0; i <= o.mask; i++)
        if (o.cnt[i] && F(cm_add)(m, o.keys[i], o.cnt[i], o.ev[i])) return -3;
    F(cm_free)(&o);
    return 0;
}
/* count += add, event = min (count 0 = empty slot: adds are >= 1) */
static int F(cm_add)(F(cmap) *m, KEY key, uint32_t add, uint64_t ev) {
    uint64_t h = KHASH(key) & m->mask;
    while (m->cnt[h]) {
        if (m->keys[h] == key) {
            m->cnt[h] += add;
            if (ev < m->ev[h]) m->ev[h] = ev;
            return 0;
        }
        h = (h + 1) & m->mask;
    }
    m->keys[h] = key;
    m->cnt[h] = add;
    m->ev[h] = ev;
    if (2 * ++m->n > m->mask) return F(cm_grow)(m);
    return 0;
}

typedef struct {
    uint64_t ev;
    KEY key;
    uint32_t cnt;
} F(entry);

typedef struct {
    const char *buf;
    const uint64_t *offsets;
    uint64_t r0, r1, npos;
    int k, nparts, rc;
    F(cmap) *parts; /* nparts maps of this map thread */
    char err[256];
} F(mapjob);

static inline int F(part_of)(KEY key, int nparts) { return (int)((KHASH(key) >> 40) % (uint64_t)nparts); }

static void *F(map_thread)(void *arg) {
    F(mapjob) *j = (F(mapjob) *)arg;
    int rc = 0;
    const int k = j->k;
    const KEY mask = F(kmask)(k);
    static const int comp[4] = {3, 2, 1, 0};
    for (int p = 0; p < j->nparts; p++)
        if ((rc = F(cm_init)(&j->parts[p], 1 << 12))) goto fail;
    for (uint64_t r = j->r0; r < j->r1; r++) {
        const unsigned char *s = (const unsigned char *)j->buf + j->offsets[r];
        uint64_t len = j->offsets[r + 1] - j->offsets[r], local = 0;
        SEGMENTS(r, s, len, k, {
            j->npos += seglen - k + 1;
            for (int tw = 0; tw < 2; tw++) { /* ref_spark.py:78 fwd_list, :81-83 rev_list */
                KEY code = 0;
                for (uint64_t t = 0; t < seglen; t++) {
                    const int b = tw ? comp[base_code(seg[seglen - 1 - t])] : base_code(seg[t]);
                    code = ((code << 2) | (KEY)b) & mask;
                    if (t + 1 >= (uint64_t)k) {
                        if ((rc = F(cm_add)(&j->parts[F(part_of)(code, j->nparts)], code, 1, (r << 32) | local)))
                            goto fail;
                        local++;
                    }
                }
            }
        });
    }
fail:
    if (rc == -2) memcpy(j->err, g_err, sizeof j->err);
    j->rc = rc;
    return NULL;
}

typedef struct {
    F(mapjob) *maps;
    int nmaps, part, rc;
    long long limit;
    F(entry) *out;
    uint64_t n;
} F(redjob);

static int F(ev_cmp)(const void *a, const void *b) {
    const uint64_t x = ((const F(entry) *)a)->ev, y = ((const F(entry) *)b)->ev;
    return x < y ? -1 : x > y;
}

/* reduceByKey (ref_spark.py:84) for one partition, then the solid filter (build:37-39) and the
 * partition's entries in event order */
static void *F(reduce_thread)(void *arg) {
    F(redjob) *j = (F(redjob) *)arg;
    F(cmap) acc;
    uint64_t est = 0;
    for (int t = 0; t < j->nmaps; t++) est += j->maps[t].parts[j->part].n;
    if ((j->rc = F(cm_init)(&acc, est / 2 + 16))) return NULL;
    for (int t = 0; t < j->nmaps; t++) {
        F(cmap) *m = &j->maps[t].parts[j->part];
        for (uint64_t i = 0; i <= m->mask; i++)
            if (m->cnt[i] && (j->rc = F(cm_add)(&acc, m->keys[i], m->cnt[i], m->ev[i]))) goto done;
        F(cm_free)(m);
    }
    j->out = (F(entry) *)malloc((acc.n + 1) * sizeof(F(entry)));
    if (!j->out) {
        j->rc = -3;
        goto done;
    }
    for (uint64_t i = 0; i <= acc.mask; i++)
        if (acc.cnt[i] && (long long)acc.cnt[i] > j->limit) {
            j->out[j->n].ev = acc.ev[i];
            j->out[j->n].key = acc.keys[i];
            j->out[j->n].cnt = acc.cnt[i];
            j->n++;
        }
    qsort(j->out, j->n, sizeof(F(entry)), F(ev_cmp));
done:
    F(cm_free)(&acc);
    return NULL;
}

static int F(assemble_mt)(const char *buf, const uint64_t *offsets, uint64_t nreads, int k, int limit,
                          unsigned flags, int threads, oracle_result *out) {
    int rc = 0;
    const int T = threads < 1 ? 1 : threads > 256 ? 256 : threads;
    F(mapjob) *maps = (F(mapjob) *)calloc(T, sizeof(F(mapjob)));
    F(redjob) *reds = (F(redjob) *)calloc(T, sizeof(F(redjob)));
    pthread_t *th = (pthread_t *)calloc(T, sizeof(pthread_t));
    uint64_t *head = (uint64_t *)calloc(T, sizeof(uint64_t));
    F(omap) d;
    memset(&d, 0, sizeof d);
    if (!maps || !reds || !th || !head) {
        rc = -3;
        goto fail;
    }
    for (int t = 0; t < T; t++) {
        maps[t].buf = buf;
        maps[t].offsets = offsets;
        maps[t].r0 = nreads * (uint64_t)t / (uint64_t)T;
        maps[t].r1 = nreads * (uint64_t)(t + 1) / (uint64_t)T;
        maps[t].k = k;
        maps[t].nparts = T;
        maps[t].parts = (F(cmap) *)calloc(T, sizeof(F(cmap)));
        if (!maps[t].parts) {
            rc = -3;
            goto fail;
        }
    }
    for (int t = 0; t < T; t++) pthread_create(&th[t], NULL, F(map_thread), &maps[t]);
    for (int t = 0; t < T; t++) pthread_join(th[t], NULL);
    for (int t = 0; t < T; t++) {
        out->n_positions += maps[t].npos;
        if (maps[t].rc && !rc) {
            rc = maps[t].rc;
            if (rc == -2) memcpy(g_err, maps[t].err, sizeof g_err);
        }
    }
    if (rc) goto fail;
    for (int p = 0; p < T; p++) {
        reds[p].maps = maps;
        reds[p].nmaps = T;
        reds[p].part = p;
        reds[p].limit = limit;
        pthread_create(&th[p], NULL, F(reduce_thread), &reds[p]);
    }
    for (int p = 0; p < T; p++) pthread_join(th[p], NULL);
    for (int p = 0; p < T; p++)
        if (reds[p].rc) rc = reds[p].rc;
    if (rc) goto fail;
    /* merge the partitions by event: build()'s dict order */
    {
        uint64_t total = 0;
        for (int p = 0; p < T; p++) total += reds[p].n;
        if ((rc = F(om_init)(&d, total + 16))) goto fail;
        for (uint64_t i = 0; i < total; i++) {
            int best = -1;
            for (int p = 0; p < T; p++)
                if (head[p] < reds[p].n && (best < 0 || reds[p].out[head[p]].ev < reds[best].out[head[best]].ev))
                    best = p;
            const F(entry) *e = &reds[best].out[head[best]++];
            if ((rc = F(om_add)(&d, e->key, e->cnt))) goto fail;
        }
    }
fail:
    if (maps)
        for (int t = 0; t < T; t++) {
            if (maps[t].parts)
                for (int p = 0; p < T; p++) F(cm_free)(&maps[t].parts[p]);
            free(maps[t].parts);
        }
    if (reds)
        for (int p = 0; p < T; p++) free(reds[p].out);
    free(maps);
    free(reds);
    free(th);
    free(head);
    if (rc) {
        F(om_free)(&d);
        if (rc == -3) snprintf(g_err, sizeof g_err, "out of memory");
        return rc;
    }
    return F(all_contigs)(&d, k, flags, out);
}

#undef SEGMENTS
#undef F
#undef CAT
#undef CAT2
