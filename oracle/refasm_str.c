/*
 * oracle/refasm_str.c -- TEST INFRASTRUCTURE ONLY (see refasm.c).
 *
 * The literal restatement of the reference CPU assembler on byte strings, for reads holding
 * bytes other than A/C/G/T/N (lowercase, IUPAC codes, soft-masked FASTA):
 *   /root/reference/src/referenceassembler/referenceAssembler.py
 *     twin:7-10      complement only uppercase A/C/G/T, every other byte is kept (its own
 *                    complement), then reverse
 *     kmers:12-14    every window seq[i:i+k]
 *     fw/bw:16-22    extend by the four uppercase bases only
 *     build:25-42    read.split('N') (uppercase N only), forward windows then the windows of
 *                    twin(segment), d[km] += 1; delete d[x] <= limit; insertion order kept
 *     get_contig:47-56, get_contig_forward:59-77, all_contigs:79-111 (heads / tails as dicts:
 *                    a later contig with the same head k-mer replaces an earlier one)
 * The k-mers are k-byte strings in an insertion-ordered open-addressing map -- no 2-bit code,
 * so no alphabet limit.  refasm.c dispatches here when a read holds such a byte.
 *
 * One deviation, where the reference has no answer: with opaque symbols a forward walk can
 * enter a cycle that contains neither its start nor the start's twin, and
 * get_contig_forward:61-75 then never returns; here such a walk fails the call (-4).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "refasm.h"

const char *oracle_last_error(void);
void oracle_set_error(const char *msg);

/* ---- growable byte arena ---------------------------------------------------------------- */
typedef struct {
    char *p;
    uint64_t n, cap;
} arena;

static int ar_reserve(arena *a, uint64_t add) {
    if (a->n + add <= a->cap) return 0;
    uint64_t c = a->cap ? a->cap : 4096;
    while (c < a->n + add) c *= 2;
    char *q = (char *)realloc(a->p, c);
    if (!q) return -1;
    a->p = q;
    a->cap = c;
    return 0;
}

/* ---- insertion-ordered map: k-byte string -> int64 value --------------------------------- */
typedef struct {
    int k;
    arena keys;        /* entry i's key at keys.p + i * k */
    int64_t *val;      /* per entry */
    uint8_t *live;     /* per entry (deleted entries keep their slot in the order) */
    uint64_t n, ecap;  /* entries */
    uint64_t *slot;    /* hash slots: entry index + 1, 0 = empty */
    uint64_t scap;
} smap;

static uint64_t shash(const char *s, int k) {
    uint64_t h = 0x9E3779B97F4A7C15ull;
    for (int i = 0; i < k; i++) {
        h ^= (unsigned char)s[i];
        h *= 0x100000001B3ull;
        h ^= h >> 29;
    }
    return h;
}

static int sm_init(smap *m, int k) {
    memset(m, 0, sizeof *m);
    m->k = k;
    m->scap = 1024;
    m->slot = (uint64_t *)calloc(m->scap, 8);
    return m->slot ? 0 : -1;
}

static void sm_free(smap *m) {
    free(m->keys.p);
    free(m->val);
    free(m->live);
    free(m->slot);
    memset(m, 0, sizeof *m);
}

static int64_t sm_find(const smap *m, const char *s) {
    uint64_t h = shash(s, m->k) & (m->scap - 1);
    for (;;) {
        const uint64_t e = m->slot[h];
        if (!e) return -1;
        if (memcmp(m->keys.p + (e - 1) * m->k, s, m->k) == 0) return (int64_t)(e - 1);
        h = (h + 1) & (m->scap - 1);
    }
}

static int sm_grow(smap *m) {
    uint64_t nc = m->scap * 2;
    uint64_t *ns = (uint64_t *)calloc(nc, 8);
    if (!ns) return -1;
    for (uint64_t i = 0; i < m->scap; i++) {
        const uint64_t e = m->slot[i];
        if (!e) continue;
        uint64_t h = shash(m->keys.p + (e - 1) * m->k, m->k) & (nc - 1);
        while (ns[h]) h = (h + 1) & (nc - 1);
        ns[h] = e;
    }
    free(m->slot);
    m->slot = ns;
    m->scap = nc;
    return 0;
}

/* entry of s, inserted (value v0, live) at the end of the order if absent; -1 out of memory */
static int64_t sm_get(smap *m, const char *s, int64_t v0) {
    int64_t e = sm_find(m, s);
    if (e >= 0) return e;
    if (2 * (m->n + 1) > m->scap && sm_grow(m)) return -1;
    if (m->n == m->ecap) {
        uint64_t c = m->ecap ? 2 * m->ecap : 1024;
        int64_t *v = (int64_t *)realloc(m->val, c * 8);
        if (!v) return -1;
        m->val = v;
        uint8_t *l = (uint8_t *)realloc(m->live, c);
        if (!l) return -1;
        m->live = l;
        m->ecap = c;
    }
    if (ar_reserve(&m->keys, (uint64_t)m->k)) return -1;
    memcpy(m->keys.p + m->n * m->k, s, m->k);
    m->keys.n += m->k;
    m->val[m->n] = v0;
    m->live[m->n] = 1;
    uint64_t h = shash(s, m->k) & (m->scap - 1);
    while (m->slot[h]) h = (h + 1) & (m->scap - 1);
    m->slot[h] = m->n + 1;
    return (int64_t)m->n++;
}

static int sm_has(const smap *m, const char *s) {
    const int64_t e = sm_find(m, s);
    return e >= 0 && m->live[e];
}

/* ---- string algebra ---------------------------------------------------------------------- */
static char comp(char c) {
    switch (c) {
    case 'A': return 'T';
    case 'C': return 'G';
    case 'G': return 'C';
    case 'T': return 'A';
    default: return c;  /* twin:8-10: complement.get(base, base) */
    }
}

static void twin_s(const char *s, int n, char *out) {
    for (int i = 0; i < n; i++) out[i] = comp(s[n - 1 - i]);
}

static const char ACGT[4] = {'A', 'C', 'G', 'T'};

/* fw(km)[b] = km[1:] + ACGT[b] */
static void fw_s(const char *km, int k, int b, char *out) {
    memcpy(out, km + 1, k - 1);
    out[k - 1] = ACGT[b];
}
/* bw(km)[b] = ACGT[b] + km[:-1] */
static void bw_s(const char *km, int k, int b, char *out) {
    out[0] = ACGT[b];
    memcpy(out + 1, km, k - 1);
}

typedef struct {
    char *p;  /* nodes, k bytes each */
    uint64_t n, cap;
} klist;

static int kl_push(klist *l, const char *s, int k) {
    if (l->n == l->cap) {
        uint64_t c = l->cap ? 2 * l->cap : 64;
        char *q = (char *)realloc(l->p, c * k);
        if (!q) return -1;
        l->p = q;
        l->cap = c;
    }
    memcpy(l->p + l->n * k, s, k);
    l->n++;
    return 0;
}

/* get_contig_forward:59-77; 0 ok, -3 no memory, -4 a walk that does not return */
static int contig_forward(const smap *d, uint64_t nlive, const char *km, int k, klist *c) {
    char *tk = (char *)malloc(3 * (size_t)k), *y = tk + k, *z = tk + 2 * k;
    if (!tk) return -3;
    twin_s(km, k, tk);
    c->n = 0;
    if (kl_push(c, km, k)) { free(tk); return -3; }
    int rc = 0;
    for (;;) {
        const char *last = c->p + (c->n - 1) * k;
        int cnt = 0, first = -1;
        for (int b = 0; b < 4; b++) {
            fw_s(last, k, b, y);
            if (sm_has(d, y)) {
                if (first < 0) first = b;
                cnt++;
            }
        }
        if (cnt != 1) break;
        fw_s(last, k, first, y);  /* cand */
        if (memcmp(y, km, k) == 0 || memcmp(y, tk, k) == 0) break;  /* cycles, Moebius */
        twin_s(last, k, z);
        if (memcmp(y, z, k) == 0) break;  /* hairpin */
        int nb = 0;
        for (int b = 0; b < 4; b++) {
            bw_s(y, k, b, z);
            nb += sm_has(d, z);
        }
        if (nb != 1) break;
        if (c->n > nlive + 1) { rc = -4; break; }  /* the reference would loop forever */
        if (kl_push(c, y, k)) { rc = -3; break; }
    }
    free(tk);
    return rc;
}

static int append_out(arena *chars, uint64_t **offs, uint64_t *noff, uint64_t *cap, const char *s, uint64_t n) {
    if (ar_reserve(chars, n)) return -1;
    memcpy(chars->p + chars->n, s, n);
    chars->n += n;
    if (*noff == *cap) {
        uint64_t c = *cap ? 2 * *cap : 1024;
        uint64_t *q = (uint64_t *)realloc(*offs, c * 8);
        if (!q) return -1;
        *offs = q;
        *cap = c;
    }
    (*offs)[(*noff)++] = chars->n;
    return 0;
}

int oracle_assemble_str(const char *buf, const uint64_t *offsets, uint64_t nreads, int k, int limit,
                        unsigned flags, oracle_result *out) {
    memset(out, 0, sizeof(*out));
    if (k < 1) { oracle_set_error("k out of range"); return -1; }
    smap d = {0}, done = {0}, heads = {0}, tails = {0};
    int rc = -3;
    klist cf = {0}, cb = {0}, cc = {0};
    arena chars = {0}, tmp = {0};
    uint64_t *coff = NULL, ncoff = 0, ccap = 0;
    char *twk = (char *)malloc(2 * (size_t)k + 2), *w2 = twk + k;
    if (!twk || sm_init(&d, k) || sm_init(&done, k) || sm_init(&heads, k) || sm_init(&tails, k)) goto out;

    /* build:25-42 */
    for (uint64_t r = 0; r < nreads; r++) {
        const char *s = buf + offsets[r];
        const uint64_t len = offsets[r + 1] - offsets[r];
        uint64_t p = 0;
        while (p <= len) {  /* read.split('N'): segments between uppercase N */
            uint64_t q = p;
            while (q < len && s[q] != 'N') q++;
            const uint64_t m = q - p;
            if (m >= (uint64_t)k) {
                out->n_positions += m - k + 1;
                for (uint64_t i = 0; i + k <= m; i++) {
                    const int64_t e = sm_get(&d, s + p + i, 0);
                    if (e < 0) goto out;
                    d.val[e]++;
                }
                tmp.n = 0;
                if (ar_reserve(&tmp, m)) goto out;
                twin_s(s + p, (int)m, tmp.p);
                for (uint64_t i = 0; i + k <= m; i++) {
                    const int64_t e = sm_get(&d, tmp.p + i, 0);
                    if (e < 0) goto out;
                    d.val[e]++;
                }
            }
            p = q + 1;
        }
    }
    uint64_t nlive = 0;
    for (uint64_t i = 0; i < d.n; i++) {
        if (d.val[i] <= limit) d.live[i] = 0;  /* d1 = [x for x in d if d[x] <= limit]; del */
        nlive += d.live[i];
    }
    out->n_dict = nlive;
    if (flags & ORACLE_WANT_DICT) {
        out->dict_kmers = (char *)malloc(nlive * k + 1);
        out->dict_counts = (uint32_t *)malloc(nlive * 4 + 4);
        if (!out->dict_kmers || !out->dict_counts) goto out;
        uint64_t j = 0;
        for (uint64_t i = 0; i < d.n; i++)
            if (d.live[i]) {
                memcpy(out->dict_kmers + j * k, d.keys.p + i * k, k);
                out->dict_counts[j++] = (uint32_t)d.val[i];
            }
    }

    /* all_contigs:79-88 */
    if (append_out(&chars, &coff, &ncoff, &ccap, "", 0)) goto out;  /* offsets[0] = 0 */
    for (uint64_t i = 0; i < d.n; i++) {
        if (!d.live[i]) continue;
        const char *x = d.keys.p + i * k;
        if (sm_has(&done, x)) continue;
        int e = contig_forward(&d, nlive, x, k, &cf);
        if (!e) {
            twin_s(x, k, twk);
            e = contig_forward(&d, nlive, twk, k, &cb);
        }
        if (e) {
            rc = e;
            if (e == -4) oracle_set_error("a contig walk enters a cycle without its start (the reference loops forever)");
            goto out;
        }
        /* get_contig:50-55: km in fw(c_fw[-1]) ? */
        const char *last = cf.p + (cf.n - 1) * k;
        int cyc = 0;
        for (int b = 0; b < 4 && !cyc; b++) {
            fw_s(last, k, b, w2);
            cyc = memcmp(w2, x, k) == 0;
        }
        cc.n = 0;
        if (!cyc)
            for (uint64_t j = cb.n - 1; j >= 1; j--) {  /* [twin(x) for x in c_bw[-1:0:-1]] */
                twin_s(cb.p + j * k, k, twk);
                if (kl_push(&cc, twk, k)) goto out;
            }
        for (uint64_t j = 0; j < cf.n; j++)
            if (kl_push(&cc, cf.p + j * k, k)) goto out;
        /* contig_to_string:44-45 */
        tmp.n = 0;
        if (ar_reserve(&tmp, (uint64_t)k + cc.n)) goto out;
        memcpy(tmp.p, cc.p, k);
        for (uint64_t j = 1; j < cc.n; j++) tmp.p[k - 1 + j] = cc.p[j * k + k - 1];
        if (append_out(&chars, &coff, &ncoff, &ccap, tmp.p, (uint64_t)k - 1 + cc.n)) goto out;
        for (uint64_t j = 0; j < cc.n; j++) {
            if (sm_get(&done, cc.p + j * k, 0) < 0) goto out;
            twin_s(cc.p + j * k, k, twk);
            if (sm_get(&done, twk, 0) < 0) goto out;
        }
    }
    const uint64_t nc = ncoff - 1;
    out->n_contigs = nc;

    /* all_contigs:90-109 */
    for (uint64_t i = 0; i < nc; i++) {
        const char *x = chars.p + coff[i];
        const uint64_t n = coff[i + 1] - coff[i];
        int64_t e = sm_get(&heads, x, 0);  /* heads[x[:k]] = (i, '+') */
        if (e < 0) goto out;
        heads.val[e] = 2 * (int64_t)i;
        twin_s(x + n - k, k, twk);        /* tails[twin(x[-k:])] = (i, '-') */
        e = sm_get(&tails, twk, 0);
        if (e < 0) goto out;
        tails.val[e] = 2 * (int64_t)i + 1;
    }
    out->link_offsets = (uint64_t *)malloc((2 * nc + 1) * 8);
    if (!out->link_offsets) goto out;
    uint64_t nl = 0, lcap = 0;
    int64_t *lk = NULL;
    out->link_offsets[0] = 0;
    for (uint64_t i = 0; i < nc; i++) {
        const char *x = chars.p + coff[i];
        const uint64_t n = coff[i + 1] - coff[i];
        for (int side = 0; side < 2; side++) {
            if (side == 0) memcpy(twk, x + n - k, k);
            else twin_s(x, k, twk);
            for (int b = 0; b < 4; b++) {
                fw_s(twk, k, b, w2);
                int64_t e[2] = {sm_find(&heads, w2), sm_find(&tails, w2)};
                for (int t = 0; t < 2; t++) {
                    if (e[t] < 0) continue;
                    if (nl == lcap) {
                        lcap = lcap ? 2 * lcap : 1024;
                        int64_t *q = (int64_t *)realloc(lk, lcap * 8);
                        if (!q) { free(lk); goto out; }
                        lk = q;
                    }
                    lk[nl++] = (t == 0 ? heads.val : tails.val)[e[t]];
                }
            }
            out->link_offsets[2 * i + side + 1] = nl;
        }
    }
    out->links = lk ? lk : (int64_t *)malloc(8);
    out->contig_offsets = (uint64_t *)malloc((nc + 1) * 8);
    out->contig_chars = (char *)malloc(chars.n + 1);
    if (!out->links || !out->contig_offsets || !out->contig_chars) goto out;
    out->contig_offsets[0] = 0;
    for (uint64_t i = 0; i < nc; i++) out->contig_offsets[i + 1] = coff[i + 1];
    memcpy(out->contig_chars, chars.p, chars.n);
    rc = 0;
out:
    if (rc == -3) oracle_set_error("out of memory");
    sm_free(&d);
    sm_free(&done);
    sm_free(&heads);
    sm_free(&tails);
    free(cf.p);
    free(cb.p);
    free(cc.p);
    free(chars.p);
    free(tmp.p);
    free(coff);
    free(twk);
    return rc;
}
