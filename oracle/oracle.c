/*
 * oracle.c -- CPU restatement of the reference BFS path.  TEST INFRASTRUCTURE ONLY.
 * See oracle.h for what each function restates and how the oracle is pinned.
 * Never linked into the product (libbfsx.so).
 */
#define _GNU_SOURCE
#include "oracle.h"

#include <errno.h>
#include <limits.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

void orc_free(void *p) { free(p); }

/* ------------------------------------------------------------------------------------------
 * File reading helpers
 * ---------------------------------------------------------------------------------------- */
static int read_file(const char *path, char **buf, size_t *len) {
    FILE *f = fopen(path, "rb");
    if (!f) return ORC_E_IO;
    if (fseek(f, 0, SEEK_END) != 0) { fclose(f); return ORC_E_IO; }
    long sz = ftell(f);
    if (sz < 0) { fclose(f); return ORC_E_IO; }
    rewind(f);
    char *b = (char *)malloc((size_t)sz + 1);
    if (!b) { fclose(f); return ORC_E_OOM; }
    size_t got = fread(b, 1, (size_t)sz, f);
    fclose(f);
    if (got != (size_t)sz) { free(b); return ORC_E_IO; }
    b[sz] = 0;
    *buf = b;
    *len = (size_t)sz;
    return ORC_OK;
}

/* java.io.BufferedReader.readLine: a line ends at '\n', '\r' or "\r\n"; returns 0 at EOF. */
static int next_line(const char *buf, size_t len, size_t *pos, const char **ls, size_t *ll) {
    if (*pos >= len) return 0;
    size_t s = *pos, e = s;
    while (e < len && buf[e] != '\n' && buf[e] != '\r') e++;
    *ls = buf + s;
    *ll = e - s;
    if (e < len) e += (buf[e] == '\r' && e + 1 < len && buf[e + 1] == '\n') ? 2 : 1;
    *pos = e;
    return 1;
}

/* InputStreamReader (UTF-8, the Linux platform charset; GraphFileUtil.java:46) turns the token's bytes
 * into UTF-16 chars: a malformed sequence becomes U+FFFD, a 4-byte sequence a surrogate pair.  Writes
 * at most n chars to w and returns their count. */
static size_t utf8_to_utf16(const unsigned char *s, size_t n, uint32_t *w) {
    size_t i = 0, k = 0;
    while (i < n) {
        const unsigned c = s[i];
        int len = c < 0x80 ? 1 : (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : (c >> 3) == 30 ? 4 : 0;
        uint32_t cp = len == 1 ? c : len == 2 ? (c & 31u) : len == 3 ? (c & 15u) : (c & 7u);
        int ok = len > 0 && i + (size_t)len <= n;
        for (int j = 1; ok && j < len; j++) {
            if ((s[i + j] & 0xC0u) != 0x80u) ok = 0;
            else cp = (cp << 6) | (s[i + j] & 0x3Fu);
        }
        if (ok && ((len == 2 && cp < 0x80) || (len == 3 && (cp < 0x800 || (cp >= 0xD800 && cp <= 0xDFFF))) ||
                   (len == 4 && (cp < 0x10000 || cp > 0x10FFFF))))
            ok = 0;
        if (!ok) {
            w[k++] = 0xFFFD;
            i++;
            continue;
        }
        if (cp >= 0x10000) {
            w[k++] = 0xD800 + ((cp - 0x10000) >> 10);
            w[k++] = 0xDC00 + ((cp - 0x10000) & 0x3FF);
        } else {
            w[k++] = cp;
        }
        i += (size_t)len;
    }
    return k;
}

/* Character.digit(ch, 10) on a UTF-16 char: the Unicode Nd digits of the BMP that Java 8 (Unicode 6.2)
 * knows, one entry per block of ten (Character.getType(ch) == DECIMAL_DIGIT_NUMBER). */
static int java_char_digit(uint32_t ch) {
    static const uint32_t zero[] = {0x0030, 0x0660, 0x06F0, 0x07C0, 0x0966, 0x09E6, 0x0A66, 0x0AE6, 0x0B66,
                                    0x0BE6, 0x0C66, 0x0CE6, 0x0D66, 0x0E50, 0x0ED0, 0x0F20, 0x1040, 0x1090,
                                    0x17E0, 0x1810, 0x1946, 0x19D0, 0x1A80, 0x1A90, 0x1B50, 0x1BB0, 0x1C40,
                                    0x1C50, 0xA620, 0xA8D0, 0xA900, 0xA9D0, 0xAA50, 0xABF0, 0xFF10};
    for (size_t i = 0; i < sizeof(zero) / sizeof(zero[0]); i++)
        if (ch >= zero[i] && ch <= zero[i] + 9) return (int)(ch - zero[i]);
    return -1;
}

/* java.lang.Integer.parseInt over an exact token (no trimming): an optional '+'/'-', then chars that
 * Character.digit maps to 0..9, within int32. */
static int java_parse_int(const char *s, size_t n, int64_t *out) {
    if (n == 0) return ORC_E_PARSE;
    uint32_t stackbuf[64];
    uint32_t *w = n <= 64 ? stackbuf : (uint32_t *)malloc(n * sizeof(uint32_t));
    if (!w) return ORC_E_OOM;
    const size_t k = utf8_to_utf16((const unsigned char *)s, n, w);
    int rc = ORC_OK;
    size_t i = 0;
    int neg = 0;
    if (w[0] == '-' || w[0] == '+') {
        neg = w[0] == '-';
        i = 1;
        if (k == 1) rc = ORC_E_PARSE;
    }
    int64_t val = 0;
    for (; rc == ORC_OK && i < k; i++) {
        const int d = java_char_digit(w[i]);
        if (d < 0) rc = ORC_E_PARSE;
        val = val * 10 + d;
        if (val > 2147483648LL) rc = ORC_E_PARSE;
    }
    if (w != stackbuf) free(w);
    if (rc) return rc;
    if (neg) val = -val;
    if (val > 2147483647LL || val < -2147483648LL) return ORC_E_PARSE;
    *out = val;
    return ORC_OK;
}

/* ------------------------------------------------------------------------------------------
 * GraphFileUtil.convert (GraphFileUtil.java:45-69)
 *   line 1: vertexCount = Integer.parseInt(line)                       :48
 *   vertex 0 always exists (put before the 1..V-1 loop)                  :53-56
 *   line 2: edge count, read and ignored                                 :58-59
 *   lines 3..EOF: Splitter.on(" ").splitToList(line); parseInt(get(0)), parseInt(get(1))  :60-63
 *   vertices.get(a).addNeighbour(b); vertices.get(b).addNeighbour(a)     :64-65  (NPE if id not a vertex)
 * ---------------------------------------------------------------------------------------- */
int orc_load_graphfileutil(const char *path, int64_t *nv_out, int64_t *m_out, uint32_t **u_out,
                           uint32_t **v_out) {
    char *buf = NULL;
    size_t len = 0;
    int rc = read_file(path, &buf, &len);
    if (rc) return rc;
    size_t pos = 0;
    const char *ls;
    size_t ll;
    if (!next_line(buf, len, &pos, &ls, &ll)) { free(buf); return ORC_E_PARSE; } /* parseInt(null) */
    int64_t V;
    if (java_parse_int(ls, ll, &V)) { free(buf); return ORC_E_PARSE; }
    if (V < 0) { free(buf); return ORC_E_PARSE; } /* new HashMap<>(negative) -> IllegalArgumentException */
    int64_t nv = V > 0 ? V : 1;                    /* vertex 0 is always put (GraphFileUtil.java:53) */
    next_line(buf, len, &pos, &ls, &ll);           /* number of edges [unused] */
    size_t cap = 1024, m = 0;
    uint32_t *u = (uint32_t *)malloc(cap * sizeof(uint32_t));
    uint32_t *v = (uint32_t *)malloc(cap * sizeof(uint32_t));
    if (!u || !v) { free(buf); free(u); free(v); return ORC_E_OOM; }
    while (next_line(buf, len, &pos, &ls, &ll)) {
        /* Splitter.on(" ").splitToList: tokens separated by single spaces, empty tokens kept */
        size_t t0e = 0;
        while (t0e < ll && ls[t0e] != ' ') t0e++;
        if (t0e >= ll) { rc = ORC_E_PARSE; break; } /* pair.get(1) -> IndexOutOfBoundsException */
        const char *t1 = ls + t0e + 1;
        size_t t1n = 0;
        while (t0e + 1 + t1n < ll && t1[t1n] != ' ') t1n++;
        int64_t a, b;
        if (java_parse_int(ls, t0e, &a) || java_parse_int(t1, t1n, &b)) { rc = ORC_E_PARSE; break; }
        if (a < 0 || a >= nv || b < 0 || b >= nv) { rc = ORC_E_RANGE; break; } /* vertices.get -> null */
        if (m == cap) {
            cap *= 2;
            uint32_t *nu = (uint32_t *)realloc(u, cap * sizeof(uint32_t));
            if (nu) u = nu;
            uint32_t *nv2 = (uint32_t *)realloc(v, cap * sizeof(uint32_t));
            if (nv2) v = nv2;
            if (!nu || !nv2) { rc = ORC_E_OOM; break; }
        }
        u[m] = (uint32_t)a;
        v[m] = (uint32_t)b;
        m++;
    }
    free(buf);
    if (rc) { free(u); free(v); return rc; }
    *nv_out = nv;
    *m_out = (int64_t)m;
    *u_out = u;
    *v_out = v;
    return ORC_OK;
}

/* ------------------------------------------------------------------------------------------
 * algs4 Graph(In) (algs4.jar!/Graph.java:85-94): V = readInt, E = readInt, then exactly E pairs;
 * In.readInt = Scanner.nextInt over \p{javaWhitespace}+ (stdlib.jar!/In.java:64-65,262-264).
 * ---------------------------------------------------------------------------------------- */
static int next_ws_token(const char *buf, size_t len, size_t *pos, const char **ts, size_t *tn) {
    size_t p = *pos;
    while (p < len && (buf[p] == ' ' || buf[p] == '\t' || buf[p] == '\n' || buf[p] == '\r' ||
                       buf[p] == '\f' || buf[p] == '\v'))
        p++;
    if (p >= len) return 0;
    size_t s = p;
    while (p < len && !(buf[p] == ' ' || buf[p] == '\t' || buf[p] == '\n' || buf[p] == '\r' ||
                        buf[p] == '\f' || buf[p] == '\v'))
        p++;
    *ts = buf + s;
    *tn = p - s;
    *pos = p;
    return 1;
}

int orc_load_algs4_graph(const char *path, int64_t *nv_out, int64_t *m_out, uint32_t **u_out,
                         uint32_t **v_out) {
    char *buf = NULL;
    size_t len = 0;
    int rc = read_file(path, &buf, &len);
    if (rc) return rc;
    size_t pos = 0;
    const char *ts;
    size_t tn;
    int64_t V, E;
    if (!next_ws_token(buf, len, &pos, &ts, &tn) || java_parse_int(ts, tn, &V) || V < 0 ||
        !next_ws_token(buf, len, &pos, &ts, &tn) || java_parse_int(ts, tn, &E) || E < 0) {
        free(buf);
        return ORC_E_PARSE;
    }
    uint32_t *u = (uint32_t *)malloc((size_t)(E ? E : 1) * sizeof(uint32_t));
    uint32_t *v = (uint32_t *)malloc((size_t)(E ? E : 1) * sizeof(uint32_t));
    if (!u || !v) { free(buf); free(u); free(v); return ORC_E_OOM; }
    for (int64_t i = 0; i < E; i++) {
        int64_t a, b;
        if (!next_ws_token(buf, len, &pos, &ts, &tn) || java_parse_int(ts, tn, &a) ||
            !next_ws_token(buf, len, &pos, &ts, &tn) || java_parse_int(ts, tn, &b)) {
            rc = ORC_E_PARSE;
            break;
        }
        if (a < 0 || a >= V || b < 0 || b >= V) { rc = ORC_E_RANGE; break; } /* validateVertex */
        u[i] = (uint32_t)a;
        v[i] = (uint32_t)b;
    }
    free(buf);
    if (rc) { free(u); free(v); return rc; }
    *nv_out = V;
    *m_out = E;
    *u_out = u;
    *v_out = v;
    return ORC_OK;
}

/* ------------------------------------------------------------------------------------------
 * Neighbour sets (Vertex.neighbours is a HashSet<Integer>, Vertex.java:30; addNeighbour :74-76;
 * GraphFileUtil.java:64-65 adds both directions, so a self-loop a-a appears once in set(a)).
 * ---------------------------------------------------------------------------------------- */
static int cmp_u32(const void *a, const void *b) {
    uint32_t x = *(const uint32_t *)a, y = *(const uint32_t *)b;
    return (x > y) - (x < y);
}

int orc_build_sets(int64_t nv, int64_t m, const uint32_t *u, const uint32_t *v, int64_t **row_off_out,
                   uint32_t **col_out) {
    int64_t *deg = (int64_t *)calloc((size_t)nv + 1, sizeof(int64_t));
    if (!deg) return ORC_E_OOM;
    for (int64_t i = 0; i < m; i++) {
        deg[u[i]]++;
        if (u[i] != v[i]) deg[v[i]]++;
    }
    int64_t *off = (int64_t *)malloc(((size_t)nv + 1) * sizeof(int64_t));
    if (!off) { free(deg); return ORC_E_OOM; }
    off[0] = 0;
    for (int64_t x = 0; x < nv; x++) off[x + 1] = off[x] + deg[x];
    int64_t nnz = off[nv];
    uint32_t *col = (uint32_t *)malloc((size_t)(nnz ? nnz : 1) * sizeof(uint32_t));
    if (!col) { free(deg); free(off); return ORC_E_OOM; }
    for (int64_t x = 0; x < nv; x++) deg[x] = off[x];
    for (int64_t i = 0; i < m; i++) {
        col[deg[u[i]]++] = v[i];
        if (u[i] != v[i]) col[deg[v[i]]++] = u[i];
    }
    /* sort + unique per row, then compact */
    int64_t w = 0;
    int64_t prev_start = 0;
    for (int64_t x = 0; x < nv; x++) {
        int64_t s = prev_start, e = off[x + 1];
        prev_start = e;
        qsort(col + s, (size_t)(e - s), sizeof(uint32_t), cmp_u32);
        off[x] = w;
        for (int64_t j = s; j < e; j++)
            if (j == s || col[j] != col[j - 1]) col[w++] = col[j];
    }
    off[nv] = w;
    free(deg);
    *row_off_out = off;
    *col_out = col;
    return ORC_OK;
}

/* ------------------------------------------------------------------------------------------
 * BfsSpark map/reduce loop (BfsSpark.java:57-118), restated level-synchronously.
 *   mapper  (:66-87): a GRAY vertex u emits (n, d(u)+1, path(u)+[n], GRAY) for n in N(u) (:73-79),
 *                     is recoloured BLACK (:80), and always emits itself (:84).
 *   reducer (:90-108): dist = min (:100); colour = max ordinal (:103); path = strictly smaller
 *                     distance wins, ties -> vertex2 (:97).  The tie winner depends on Spark's
 *                     shuffle order; this restatement picks the largest emitting u, which reproduces
 *                     the outcome printed in the report (PDF p.5 Table 6: path(3) = [0, 5, 3]).
 *   terminate (:117):  continue while any vertex is GRAY after the pass.
 * ---------------------------------------------------------------------------------------- */
static inline void atomic_max_i64(int64_t *p, int64_t val) {
    int64_t cur = __atomic_load_n(p, __ATOMIC_RELAXED);
    while (cur < val &&
           !__atomic_compare_exchange_n(p, &cur, val, 0, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {
    }
}

int orc_mapreduce_bfs(int64_t nv, const int64_t *row_off, const uint32_t *col, int64_t source,
                      int32_t *dist, int64_t *parent, int8_t *color, int64_t *iter_gray,
                      int64_t *iter_emits, int64_t max_iters, int64_t *iters_out, int nthreads) {
    if (source < 0 || source >= nv) return ORC_E_RANGE;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
    int8_t *ncolor = (int8_t *)malloc((size_t)nv);
    if (!ncolor) return ORC_E_OOM;
    /* initial state: GraphFileUtil.java:53-56 */
    for (int64_t x = 0; x < nv; x++) {
        dist[x] = INT32_MAX;
        parent[x] = -1;
        color[x] = ORC_WHITE;
    }
    dist[source] = 0;
    parent[source] = source;
    color[source] = ORC_GRAY;
    int64_t iters = 0;
    int gray_left = 1;
    while (gray_left) {
        int64_t emits = 0, grays = 0;
        memcpy(ncolor, color, (size_t)nv);
        /* map: every vertex line is visited; GRAY ones expand */
#pragma omp parallel for schedule(dynamic, 1024) reduction(+ : emits)
        for (int64_t x = 0; x < nv; x++) {
            emits += 1; /* the vertex emits itself (BfsSpark.java:84) */
            if (color[x] != ORC_GRAY) continue;
            int32_t nd = dist[x] + 1;
            ncolor[x] = ORC_BLACK; /* :80, and max(BLACK, anything) = BLACK in the reducer */
            for (int64_t j = row_off[x]; j < row_off[x + 1]; j++) {
                uint32_t n = col[j];
                emits += 1;
                /* reduce: a WHITE target becomes GRAY at d+1; GRAY/BLACK targets keep their state */
                if (color[n] == ORC_WHITE) {
                    ncolor[n] = ORC_GRAY; /* idempotent write of the same value */
                    dist[n] = nd;         /* all emitters of this pass carry the same d+1 */
                    atomic_max_i64(&parent[n], x);
                }
            }
        }
        memcpy(color, ncolor, (size_t)nv);
#pragma omp parallel for reduction(+ : grays)
        for (int64_t x = 0; x < nv; x++) grays += color[x] == ORC_GRAY;
        if (iters < max_iters) {
            if (iter_gray) iter_gray[iters] = grays;
            if (iter_emits) iter_emits[iters] = emits;
        }
        iters++;
        gray_left = grays > 0; /* content.contains("GRAY") (:117) */
    }
    free(ncolor);
    if (iters_out) *iters_out = iters;
    return ORC_OK;
}

/* ------------------------------------------------------------------------------------------
 * algs4 BreadthFirstPaths.bfs (algs4.jar!/BreadthFirstPaths.java:93-111) over Graph's Bag
 * adjacency: Bag.add prepends (algs4.jar!/Bag.java:87-92), so adj(v) iterates in reverse
 * insertion order; addEdge(v,w) adds w to adj[v] then v to adj[w] (Graph.java:143-149).
 * ---------------------------------------------------------------------------------------- */
static int bag_build(int64_t nv, int64_t m, const uint32_t *u, const uint32_t *v, int64_t **off_out,
                     uint32_t **adj_out) {
    int64_t *off = (int64_t *)calloc((size_t)nv + 1, sizeof(int64_t));
    uint32_t *adj = (uint32_t *)malloc((size_t)(2 * m + 1) * sizeof(uint32_t));
    if (!off || !adj) { free(off); free(adj); return ORC_E_OOM; }
    for (int64_t i = 0; i < m; i++) {
        off[u[i] + 1]++;
        off[v[i] + 1]++;
    }
    for (int64_t x = 0; x < nv; x++) off[x + 1] += off[x];
    int64_t *cur = (int64_t *)malloc(((size_t)nv + 1) * sizeof(int64_t));
    if (!cur) { free(off); free(adj); return ORC_E_OOM; }
    /* fill each Bag back to front so that forward iteration is LIFO */
    for (int64_t x = 0; x < nv; x++) cur[x] = off[x + 1];
    for (int64_t i = 0; i < m; i++) {
        adj[--cur[u[i]]] = v[i];
        adj[--cur[v[i]]] = u[i];
    }
    free(cur);
    *off_out = off;
    *adj_out = adj;
    return ORC_OK;
}

int64_t orc_algs4_adj(int64_t nv, int64_t m, const uint32_t *u, const uint32_t *v, int64_t x,
                      uint32_t *out, int64_t cap) {
    int64_t *off;
    uint32_t *adj;
    if (x < 0 || x >= nv || bag_build(nv, m, u, v, &off, &adj)) return -1;
    int64_t k = 0;
    for (int64_t j = off[x]; j < off[x + 1] && k < cap; j++) out[k++] = adj[j];
    free(off);
    free(adj);
    return k;
}

int orc_algs4_bfs(int64_t nv, int64_t m, const uint32_t *u, const uint32_t *v, int64_t source,
                  int32_t *dist, int64_t *edge_to) {
    if (source < 0 || source >= nv) return ORC_E_RANGE;
    int64_t *off;
    uint32_t *adj;
    int rc = bag_build(nv, m, u, v, &off, &adj);
    if (rc) return rc;
    uint32_t *q = (uint32_t *)malloc((size_t)nv * sizeof(uint32_t));
    uint8_t *marked = (uint8_t *)calloc((size_t)nv, 1);
    if (!q || !marked) { free(off); free(adj); free(q); free(marked); return ORC_E_OOM; }
    for (int64_t x = 0; x < nv; x++) { dist[x] = INT32_MAX; edge_to[x] = -1; }
    int64_t qh = 0, qt = 0;
    dist[source] = 0;
    edge_to[source] = source;
    marked[source] = 1;
    q[qt++] = (uint32_t)source;
    while (qh < qt) {
        uint32_t x = q[qh++];
        for (int64_t j = off[x]; j < off[x + 1]; j++) {
            uint32_t w = adj[j];
            if (!marked[w]) {
                edge_to[w] = x;
                dist[w] = dist[x] + 1;
                marked[w] = 1;
                q[qt++] = w;
            }
        }
    }
    free(off); free(adj); free(q); free(marked);
    return ORC_OK;
}

int orc_csr_bfs(int64_t nv, const int64_t *row_off, const uint32_t *col, int64_t source, int32_t *dist,
                int64_t *parent) {
    if (source < 0 || source >= nv) return ORC_E_RANGE;
    uint32_t *q = (uint32_t *)malloc((size_t)nv * sizeof(uint32_t));
    if (!q) return ORC_E_OOM;
    for (int64_t x = 0; x < nv; x++) { dist[x] = INT32_MAX; if (parent) parent[x] = -1; }
    int64_t qh = 0, qt = 0;
    dist[source] = 0;
    if (parent) parent[source] = source;
    q[qt++] = (uint32_t)source;
    while (qh < qt) {
        uint32_t x = q[qh++];
        int32_t nd = dist[x] + 1;
        for (int64_t j = row_off[x]; j < row_off[x + 1]; j++) {
            uint32_t w = col[j];
            if (dist[w] == INT32_MAX) {
                dist[w] = nd;
                if (parent) parent[w] = x;
                q[qt++] = w;
            }
        }
    }
    free(q);
    return ORC_OK;
}

/* ------------------------------------------------------------------------------------------
 * Validation: BreadthFirstPaths.check (algs4.jar!/BreadthFirstPaths.java:171-212) plus the
 * Graph500 parent-tree rules (tree edges are graph edges, levels differ by one along every edge,
 * reachability agrees across every edge).
 * ---------------------------------------------------------------------------------------- */
static int has_edge(const int64_t *row_off, const uint32_t *col, uint32_t a, uint32_t b) {
    int64_t lo = row_off[a], hi = row_off[a + 1];
    while (lo < hi) { /* rows are sorted */
        int64_t mid = lo + (hi - lo) / 2;
        if (col[mid] < b) lo = mid + 1;
        else hi = mid;
    }
    return lo < row_off[a + 1] && col[lo] == b;
}

int orc_validate(int64_t nv, const int64_t *row_off, const uint32_t *col, int64_t source,
                 const int32_t *dist, const int64_t *parent) {
    if (source < 0 || source >= nv) return -1;
    if (dist[source] != 0 || parent[source] != source) return -1;
    int bad = 0;
#pragma omp parallel for schedule(dynamic, 4096) reduction(min : bad)
    for (int64_t x = 0; x < nv; x++) {
        int r = 0;
        if (dist[x] == INT32_MAX) {
            if (parent[x] != -1) r = -5;
        } else if (x != source) {
            int64_t p = parent[x];
            if (p < 0 || p >= nv) r = -5;
            else if (dist[p] == INT32_MAX || dist[x] != dist[p] + 1) r = -2;
            else if (!has_edge(row_off, col, (uint32_t)p, (uint32_t)x)) r = -3;
        }
        if (!r) {
            for (int64_t j = row_off[x]; j < row_off[x + 1]; j++) {
                uint32_t y = col[j];
                int ra = dist[x] != INT32_MAX, rb = dist[y] != INT32_MAX;
                if (ra != rb) { r = -4; break; }
                if (ra) {
                    int64_t dd = (int64_t)dist[x] - (int64_t)dist[y];
                    if (dd > 1 || dd < -1) { r = -4; break; }
                }
            }
        }
        if (r < bad) bad = r;
    }
    return bad;
}

/* ------------------------------------------------------------------------------------------
 * Kronecker generator: Graph500 spec recipe (A,B,C,D = .57,.19,.19,.05) with an integer,
 * counter-based RNG so that the GPU generator and this one agree bit for bit:
 *   r(k, ib) = mix64((k << 6 | ib) ^ mix64(seed))      splitmix64 finaliser
 *   ii = hi32(r) > T_ab ; jj = lo32(r) > (ii ? T_cnorm : T_anorm)
 *   i |= ii << ib ; j |= jj << ib        for ib in [0, scale)
 *   u = perm(i), v = perm(j)             bijective scramble of [0, 2^scale)
 * ---------------------------------------------------------------------------------------- */
static inline uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

void orc_kronecker_thresholds(uint32_t *t_ab, uint32_t *t_a_norm, uint32_t *t_c_norm) {
    /* ab = A+B = 0.76; a_norm = A/(A+B) = 57/76; c_norm = C/(1-(A+B)) = 19/24 */
    *t_ab = (uint32_t)((76ULL << 32) / 100ULL);
    *t_a_norm = (uint32_t)((57ULL << 32) / 76ULL);
    *t_c_norm = (uint32_t)((19ULL << 32) / 24ULL);
}

static inline uint64_t kron_perm(uint64_t x, int scale, uint64_t seed) {
    uint64_t mask = (scale >= 64) ? ~0ULL : ((1ULL << scale) - 1);
    uint64_t a1 = (mix64(seed ^ 0xA5A5A5A5A5A5A5A5ULL) | 1ULL) & mask;
    uint64_t c1 = mix64(seed ^ 0x5A5A5A5A5A5A5A5AULL) & mask;
    uint64_t a2 = (mix64(seed ^ 0x3C3C3C3C3C3C3C3CULL) | 1ULL) & mask;
    uint64_t c2 = mix64(seed ^ 0xC3C3C3C3C3C3C3C3ULL) & mask;
    int s1 = scale / 2 + 1, s2 = scale / 3 + 1;
    x = (x * a1 + c1) & mask;
    x ^= x >> s1;
    x = (x * a2 + c2) & mask;
    x ^= x >> s2;
    x = (x * a1 + c2) & mask;
    return x;
}

void orc_kronecker(int scale, int edgefactor, uint64_t seed, uint32_t *u, uint32_t *v) {
    uint32_t t_ab, t_an, t_cn;
    orc_kronecker_thresholds(&t_ab, &t_an, &t_cn);
    uint64_t m = (uint64_t)edgefactor << scale;
    uint64_t sh = mix64(seed);
#pragma omp parallel for schedule(static)
    for (int64_t k = 0; k < (int64_t)m; k++) {
        uint64_t i = 0, j = 0;
        for (int ib = 0; ib < scale; ib++) {
            uint64_t r = mix64((((uint64_t)k) << 6 | (uint64_t)ib) ^ sh);
            uint32_t r1 = (uint32_t)(r >> 32), r2 = (uint32_t)r;
            uint64_t ii = r1 > t_ab;
            uint64_t jj = r2 > (ii ? t_cn : t_an);
            i |= ii << ib;
            j |= jj << ib;
        }
        u[k] = (uint32_t)kron_perm(i, scale, seed);
        v[k] = (uint32_t)kron_perm(j, scale, seed);
    }
}

int64_t orc_mcomp(int64_t m, const uint32_t *u, const uint32_t *v, const int32_t *dist) {
    int64_t c = 0;
    (void)v;
#pragma omp parallel for reduction(+ : c)
    for (int64_t i = 0; i < m; i++) c += dist[u[i]] != INT32_MAX;
    return c;
}

/* ------------------------------------------------------------------------------------------
 * sha256 (FIPS 180-4) for the Appendix A hashes of "v d\n" lines.
 * ---------------------------------------------------------------------------------------- */
typedef struct {
    uint32_t h[8];
    uint8_t buf[64];
    uint64_t len;
    size_t fill;
} sha_ctx;

static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

#define ROR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))
static void sha_block(sha_ctx *c, const uint8_t *p) {
    uint32_t w[64];
    for (int i = 0; i < 16; i++)
        w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 | (uint32_t)p[4 * i + 2] << 8 |
               p[4 * i + 3];
    for (int i = 16; i < 64; i++) {
        uint32_t s0 = ROR(w[i - 15], 7) ^ ROR(w[i - 15], 18) ^ (w[i - 15] >> 3);
        uint32_t s1 = ROR(w[i - 2], 17) ^ ROR(w[i - 2], 19) ^ (w[i - 2] >> 10);
        w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = c->h[0], b = c->h[1], cc = c->h[2], d = c->h[3], e = c->h[4], f = c->h[5],
             g = c->h[6], h = c->h[7];
    for (int i = 0; i < 64; i++) {
        uint32_t S1 = ROR(e, 6) ^ ROR(e, 11) ^ ROR(e, 25);
        uint32_t ch = (e & f) ^ (~e & g);
        uint32_t t1 = h + S1 + ch + K256[i] + w[i];
        uint32_t S0 = ROR(a, 2) ^ ROR(a, 13) ^ ROR(a, 22);
        uint32_t mj = (a & b) ^ (a & cc) ^ (b & cc);
        uint32_t t2 = S0 + mj;
        h = g; g = f; f = e; e = d + t1; d = cc; cc = b; b = a; a = t1 + t2;
    }
    c->h[0] += a; c->h[1] += b; c->h[2] += cc; c->h[3] += d;
    c->h[4] += e; c->h[5] += f; c->h[6] += g; c->h[7] += h;
}

static void sha_init(sha_ctx *c) {
    static const uint32_t h0[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                   0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    memcpy(c->h, h0, sizeof(h0));
    c->len = 0;
    c->fill = 0;
}

static void sha_update(sha_ctx *c, const uint8_t *p, size_t n) {
    c->len += n;
    while (n) {
        size_t k = 64 - c->fill;
        if (k > n) k = n;
        memcpy(c->buf + c->fill, p, k);
        c->fill += k;
        p += k;
        n -= k;
        if (c->fill == 64) { sha_block(c, c->buf); c->fill = 0; }
    }
}

static void sha_final(sha_ctx *c, uint8_t out[32]) {
    uint64_t bits = c->len * 8;
    uint8_t pad = 0x80;
    sha_update(c, &pad, 1);
    uint8_t z = 0;
    while (c->fill != 56) sha_update(c, &z, 1);
    uint8_t lb[8];
    for (int i = 0; i < 8; i++) lb[i] = (uint8_t)(bits >> (56 - 8 * i));
    sha_update(c, lb, 8);
    for (int i = 0; i < 8; i++) {
        out[4 * i] = (uint8_t)(c->h[i] >> 24);
        out[4 * i + 1] = (uint8_t)(c->h[i] >> 16);
        out[4 * i + 2] = (uint8_t)(c->h[i] >> 8);
        out[4 * i + 3] = (uint8_t)c->h[i];
    }
}

void orc_dist_sha256(int64_t nv, const int32_t *dist, char *out_hex) {
    sha_ctx c;
    sha_init(&c);
    char line[64];
    for (int64_t x = 0; x < nv; x++) {
        int k = snprintf(line, sizeof(line), "%lld %d\n", (long long)x, dist[x]);
        sha_update(&c, (const uint8_t *)line, (size_t)k);
    }
    uint8_t d[32];
    sha_final(&c, d);
    for (int i = 0; i < 32; i++) sprintf(out_hex + 2 * i, "%02x", d[i]);
    out_hex[64] = 0;
}
