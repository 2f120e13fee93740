/*
 * orc.c — CPU oracle (TEST INFRASTRUCTURE ONLY; see orc.h for the scope and the
 * "parity unpinned" statement).
 *
 * Citations: reference paths are relative to the LiHeng/goworld tree.
 * [EXT] marks go-aoi v0.2.0 (go.mod:25), which is absent from the container;
 * those parts restate the published algorithm as written down in SURVEY.md
 * Appendix A.
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off, no fast-math: the window
 * bounds fl(c-d), fl(c+d) must be float32 round-to-nearest-even, as Go's
 * float32 Coord arithmetic is).
 */
#include "orc.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* qsort of n elements; qsort(NULL, 0, ...) is undefined behaviour (its base
 * is declared non-null), so empty and single-element arrays are left alone */
static void sort_n(void* base, size_t n, size_t size, int (*cmp)(const void*, const void*)) {
    if (n > 1) qsort(base, n, size, cmp);
}

/* ------------------------------------------------------------------------ */
/* small growable u32 set (Go map[*T]struct{} stand-in: order is irrelevant) */
typedef struct { uint32_t* a; uint32_t n, cap; } vec32;


static void v_push(vec32* v, uint32_t x) {
    if (v->n == v->cap) {
        v->cap = v->cap ? v->cap * 2 : 8;
        v->a = (uint32_t*)realloc(v->a, (size_t)v->cap * 4);
        if (!v->a) { fprintf(stderr, "orc: out of memory\n"); abort(); }
    }
    v->a[v->n++] = x;
}
static int v_del(vec32* v, uint32_t x) {
    for (uint32_t i = 0; i < v->n; ++i)
        if (v->a[i] == x) { v->a[i] = v->a[--v->n]; return 1; }
    return 0;
}
static void v_clear(vec32* v) { v->n = 0; }
static void v_free(vec32* v) { free(v->a); v->a = NULL; v->n = v->cap = 0; }

static int cmp_u32(const void* a, const void* b) {
    uint32_t x = *(const uint32_t*)a, y = *(const uint32_t*)b;
    return x < y ? -1 : x > y;
}
static int cmp_u64(const void* a, const void* b) {
    uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
    return x < y ? -1 : x > y;
}

/* ------------------------------------------------------------------------ */
/* go-aoi xzaoi node [EXT]: xPrev,xNext,yPrev,yNext,markVal (+ neighbors)    */
typedef struct { int32_t prev[2], next[2]; int32_t mark; } xznode;

typedef struct { uint64_t key; int32_t d; } rawev;   /* key = watcher<<32|target */

struct orc_space {
    int mode;
    uint32_t cap;
    float d;                       /* XZListAOIManager.aoidist [EXT]           */
    uint8_t* present;
    uint8_t* flags;                /* Entity.syncInfoFlag (Entity.go:63)        */
    uint16_t* gate;                /* client gate id, 0 = no client             */
    float* ac[2];                  /* aoi.x, aoi.y  (= Position.X, Position.Z)  */
    float *px, *py, *pz, *pyaw;    /* Entity.Position, Entity.yaw (sync data)   */
    vec32* nb;                     /* xzaoi.neighbors / relation                */
    vec32* in;                     /* Entity.InterestedIn (Entity.go:53)        */
    vec32* by;                     /* Entity.InterestedBy (Entity.go:54)        */
    xznode* node;
    int32_t head[2], tail[2];
    /* per-tick bookkeeping */
    rawev* raw; size_t nraw, capraw;
    uint64_t raw_enter, raw_leave, create_msgs, destroy_msgs;
    gw_event *enter, *leave; uint64_t n_enter, n_leave;
    gw_sync_record* rec; uint64_t n_rec;
    /* scratch */
    int32_t* seq; uint8_t* mk; uint8_t* mk2;
};

static float coordv(const orc_space* s, int ax, int32_t i) { return s->ac[ax][i]; }

/* exact reference window: other in [fl(c-d), fl(c+d)] on X and Z.
 * go-aoi xzlist Mark: minCoord := coord - aoidist; p.x >= minCoord;
 * maxCoord := coord + aoidist; p.x <= maxCoord  [EXT]                      */
int orc_in_window(float cx, float cz, float d, float ox, float oz) {
    float lox = cx - d, hix = cx + d, loz = cz - d, hiz = cz + d;
    return ox >= lox && ox <= hix && oz >= loz && oz <= hiz;
}

/* ------------------------------------------------------------------------ */
orc_space* orc_new(uint32_t capacity, float d, int mode) {
    if (!(d > 0) || capacity == 0 || mode < 0 || mode > 2) return NULL;
    orc_space* s = (orc_space*)calloc(1, sizeof(orc_space));
    s->mode = mode; s->cap = capacity; s->d = d;
    size_t n = capacity;
    s->present = (uint8_t*)calloc(n, 1);
    s->flags = (uint8_t*)calloc(n, 1);
    s->gate = (uint16_t*)calloc(n, 2);
    s->ac[0] = (float*)calloc(n, 4); s->ac[1] = (float*)calloc(n, 4);
    s->px = (float*)calloc(n, 4); s->py = (float*)calloc(n, 4);
    s->pz = (float*)calloc(n, 4); s->pyaw = (float*)calloc(n, 4);
    s->nb = (vec32*)calloc(n, sizeof(vec32));
    if (mode != ORC_SEQRULE) {
        s->in = (vec32*)calloc(n, sizeof(vec32));
        s->by = (vec32*)calloc(n, sizeof(vec32));
    }
    s->node = (xznode*)calloc(n, sizeof(xznode));
    for (size_t i = 0; i < n; ++i)
        s->node[i].prev[0] = s->node[i].prev[1] = s->node[i].next[0] = s->node[i].next[1] = -1;
    s->head[0] = s->head[1] = s->tail[0] = s->tail[1] = -1;
    s->seq = (int32_t*)malloc(n * 4);
    for (size_t i = 0; i < n; ++i) s->seq[i] = -1;
    s->mk = (uint8_t*)calloc(n, 1); s->mk2 = (uint8_t*)calloc(n, 1);
    return s;
}

void orc_free(orc_space* s) {
    if (!s) return;
    for (uint32_t i = 0; i < s->cap; ++i) {
        v_free(&s->nb[i]);
        if (s->in) { v_free(&s->in[i]); v_free(&s->by[i]); }
    }
    free(s->present); free(s->flags); free(s->gate); free(s->ac[0]); free(s->ac[1]);
    free(s->px); free(s->py); free(s->pz); free(s->pyaw);
    free(s->nb); free(s->in); free(s->by); free(s->node); free(s->raw);
    free(s->enter); free(s->leave); free(s->rec); free(s->seq); free(s->mk); free(s->mk2);
    free(s);
}

/* ------------------------------------------------------------------------ */
/* goworld glue: Entity.OnEnterAOI/OnLeaveAOI -> interest/uninterest          */
/* (Entity.go:227-246) plus GameClient.sendCreateEntity/sendDestroyEntity     */
/* message counts (GameClient.go:37-59: no message without a client).         */
static void raw_push(orc_space* s, uint32_t w, uint32_t t, int d) {
    if (s->nraw == s->capraw) {
        s->capraw = s->capraw ? s->capraw * 2 : 1024;
        s->raw = (rawev*)realloc(s->raw, s->capraw * sizeof(rawev));
    }
    s->raw[s->nraw].key = ((uint64_t)w << 32) | t;
    s->raw[s->nraw].d = d;
    s->nraw++;
}
static void on_enter_aoi(orc_space* s, uint32_t w, uint32_t t) {   /* w.OnEnterAOI(t) */
    raw_push(s, w, t, +1); s->raw_enter++;
    v_push(&s->in[w], t);            /* e.InterestedIn.Add(other)   */
    v_push(&s->by[t], w);            /* other.InterestedBy.Add(e)   */
    if (s->gate[w]) s->create_msgs++;
}
static void on_leave_aoi(orc_space* s, uint32_t w, uint32_t t) {   /* w.OnLeaveAOI(t) */
    raw_push(s, w, t, -1); s->raw_leave++;
    v_del(&s->in[w], t);             /* e.InterestedIn.Del(other)   */
    v_del(&s->by[t], w);             /* other.InterestedBy.Del(e)   */
    if (s->gate[w]) s->destroy_msgs++;
}

/* ------------------------------------------------------------------------ */
/* go-aoi xAOIList / yAOIList [EXT] — one implementation per axis (0=X, 1=Z) */
static void list_insert(orc_space* s, int ax, int32_t n) {
    xznode* N = s->node;
    float c = coordv(s, ax, n);
    N[n].prev[ax] = N[n].next[ax] = -1;
    if (s->head[ax] == -1) { s->head[ax] = s->tail[ax] = n; return; }
    int32_t p = s->head[ax];
    while (p != -1 && coordv(s, ax, p) < c) p = N[p].next[ax];   /* walk from head */
    if (p == -1) {                                              /* append at tail */
        int32_t t = s->tail[ax];
        N[t].next[ax] = n; N[n].prev[ax] = t; s->tail[ax] = n;
    } else {                                                    /* insert before p (p.c >= c) */
        int32_t pr = N[p].prev[ax];
        N[n].next[ax] = p; N[p].prev[ax] = n; N[n].prev[ax] = pr;
        if (pr != -1) N[pr].next[ax] = n; else s->head[ax] = n;
    }
}

static void list_remove(orc_space* s, int ax, int32_t n) {
    xznode* N = s->node;
    int32_t pr = N[n].prev[ax], nx = N[n].next[ax];
    if (pr != -1) { N[pr].next[ax] = nx; N[n].prev[ax] = -1; } else s->head[ax] = nx;
    if (nx != -1) { N[nx].prev[ax] = pr; N[n].next[ax] = -1; } else s->tail[ax] = pr;
}

static void list_move(orc_space* s, int ax, int32_t n, float oldc) {
    xznode* N = s->node;
    float c = coordv(s, ax, n);
    if (c > oldc) {                                   /* moving to next */
        int32_t nx = N[n].next[ax];
        if (nx == -1 || coordv(s, ax, nx) >= c) return;
        int32_t pr = N[n].prev[ax];
        if (pr != -1) N[pr].next[ax] = nx; else s->head[ax] = nx;
        N[nx].prev[ax] = pr;
        pr = nx; nx = N[nx].next[ax];
        while (nx != -1 && coordv(s, ax, nx) < c) { pr = nx; nx = N[nx].next[ax]; }
        N[pr].next[ax] = n; N[n].prev[ax] = pr;
        if (nx != -1) N[nx].prev[ax] = n; else s->tail[ax] = n;
        N[n].next[ax] = nx;
    } else {                                          /* moving to prev */
        int32_t pr = N[n].prev[ax];
        if (pr == -1 || coordv(s, ax, pr) <= c) return;
        int32_t nx = N[n].next[ax];
        if (nx != -1) N[nx].prev[ax] = pr; else s->tail[ax] = pr;
        N[pr].next[ax] = nx;
        nx = pr; pr = N[pr].prev[ax];
        while (pr != -1 && coordv(s, ax, pr) > c) { nx = pr; pr = N[pr].prev[ax]; }
        N[nx].prev[ax] = n; N[n].next[ax] = nx;
        if (pr != -1) N[pr].next[ax] = n; else s->head[ax] = n;
        N[n].prev[ax] = pr;
    }
}

static void list_mark(orc_space* s, int ax, int32_t n) {
    xznode* N = s->node;
    float c = coordv(s, ax, n);
    float lo = c - s->d;
    for (int32_t p = N[n].prev[ax]; p != -1 && coordv(s, ax, p) >= lo; p = N[p].prev[ax]) N[p].mark += 1;
    float hi = c + s->d;
    for (int32_t p = N[n].next[ax]; p != -1 && coordv(s, ax, p) <= hi; p = N[p].next[ax]) N[p].mark += 1;
}

static void add_neighbor_pair(orc_space* s, int32_t a, int32_t p) {
    /* aoi.neighbors[prev] = {}; aoi.callback.OnEnterAOI(prev.aoi);
       prev.neighbors[aoi] = {}; prev.callback.OnEnterAOI(aoi.aoi)   [EXT] */
    v_push(&s->nb[a], (uint32_t)p); on_enter_aoi(s, (uint32_t)a, (uint32_t)p);
    v_push(&s->nb[p], (uint32_t)a); on_enter_aoi(s, (uint32_t)p, (uint32_t)a);
}

static void list_get_clear_marked(orc_space* s, int32_t n) {     /* X list [EXT] */
    xznode* N = s->node;
    float c = coordv(s, 0, n);
    float lo = c - s->d;
    for (int32_t p = N[n].prev[0]; p != -1 && coordv(s, 0, p) >= lo; p = N[p].prev[0]) {
        if (N[p].mark == 2) add_neighbor_pair(s, n, p);
        N[p].mark = 0;
    }
    float hi = c + s->d;
    for (int32_t p = N[n].next[0]; p != -1 && coordv(s, 0, p) <= hi; p = N[p].next[0]) {
        if (N[p].mark == 2) add_neighbor_pair(s, n, p);
        N[p].mark = 0;
    }
}

static void list_clear_mark(orc_space* s, int32_t n) {           /* Z list [EXT] */
    xznode* N = s->node;
    float c = coordv(s, 1, n);
    float lo = c - s->d;
    for (int32_t p = N[n].prev[1]; p != -1 && coordv(s, 1, p) >= lo; p = N[p].prev[1]) N[p].mark = 0;
    float hi = c + s->d;
    for (int32_t p = N[n].next[1]; p != -1 && coordv(s, 1, p) <= hi; p = N[p].next[1]) N[p].mark = 0;
}

/* XZListAOIManager.adjust [EXT] */
static void xz_adjust(orc_space* s, int32_t n) {
    xznode* N = s->node;
    list_mark(s, 0, n);
    list_mark(s, 1, n);
    vec32* nbn = &s->nb[n];
    for (uint32_t i = 0; i < nbn->n;) {          /* for neighbor := range aoi.neighbors */
        uint32_t m = nbn->a[i];
        if (N[m].mark == 2) { N[m].mark = -2; ++i; continue; }   /* kept */
        nbn->a[i] = nbn->a[--nbn->n];             /* delete(aoi.neighbors, neighbor) */
        on_leave_aoi(s, (uint32_t)n, m);
        v_del(&s->nb[m], (uint32_t)n);            /* delete(neighbor.neighbors, aoi) */
        on_leave_aoi(s, m, (uint32_t)n);
    }
    list_get_clear_marked(s, n);
    list_clear_mark(s, n);
}

static void xz_enter(orc_space* s, int32_t n) {     /* Enter [EXT] */
    s->node[n].mark = 0;
    v_clear(&s->nb[n]);
    list_insert(s, 0, n);
    list_insert(s, 1, n);
    xz_adjust(s, n);
}
static void xz_leave(orc_space* s, int32_t n) {     /* Leave [EXT] */
    list_remove(s, 0, n);
    list_remove(s, 1, n);
    xz_adjust(s, n);
}
static void xz_moved(orc_space* s, int32_t n, float oldx, float oldz) {  /* Moved [EXT] */
    if (oldx != s->ac[0][n]) list_move(s, 0, n, oldx);
    if (oldz != s->ac[1][n]) list_move(s, 1, n, oldz);
    xz_adjust(s, n);
}

/* ------------------------------------------------------------------------ */
/* ORC_BRUTE: sequential, relation(A,b) := inWin_A(b) after each op on A     */
static void brute_adjust(orc_space* s, int32_t a) {
    uint8_t* want = s->mk;     /* want[b]: b in A's window now */
    uint8_t* have = s->mk2;    /* have[b]: b currently a neighbour */
    vec32* nba = &s->nb[a];
    for (uint32_t i = 0; i < nba->n; ++i) have[nba->a[i]] = 1;
    uint32_t nwant = 0;
    if (s->present[a]) {
        for (uint32_t b = 0; b < s->cap; ++b)
            if (b != (uint32_t)a && s->present[b] &&
                orc_in_window(s->ac[0][a], s->ac[1][a], s->d, s->ac[0][b], s->ac[1][b])) {
                want[b] = 1; ++nwant;
            }
    }
    /* leaves */
    for (uint32_t i = 0; i < nba->n;) {
        uint32_t m = nba->a[i];
        if (!want[m]) {
            nba->a[i] = nba->a[--nba->n];
            have[m] = 0;
            on_leave_aoi(s, (uint32_t)a, m);
            v_del(&s->nb[m], (uint32_t)a);
            on_leave_aoi(s, m, (uint32_t)a);
        } else ++i;
    }
    /* enters */
    if (nwant) {
        for (uint32_t b = 0; b < s->cap; ++b) {
            if (want[b] && !have[b]) {
                v_push(&s->nb[a], b); on_enter_aoi(s, (uint32_t)a, b);
                v_push(&s->nb[b], (uint32_t)a); on_enter_aoi(s, b, (uint32_t)a);
            }
            want[b] = 0;
        }
    }
    for (uint32_t i = 0; i < nba->n; ++i) have[nba->a[i]] = 0;
}

/* ------------------------------------------------------------------------ */
/* uniform grid over present entities (bulk build + SEQRULE)                 */
typedef struct { uint64_t key; uint32_t slot; } gent;
static int cmp_gent(const void* a, const void* b) {
    const gent* x = (const gent*)a; const gent* y = (const gent*)b;
    if (x->key != y->key) return x->key < y->key ? -1 : 1;
    return x->slot < y->slot ? -1 : x->slot > y->slot;
}
static int64_t cell_of(double c, double d) {
    double q = floor(c / d);
    if (q < -1073741824.0) q = -1073741824.0;
    if (q > 1073741823.0) q = 1073741823.0;
    return (int64_t)q;
}
static uint64_t cell_key(int64_t cx, int64_t cz) {
    return ((uint64_t)(cz + 2147483648LL) << 32) | (uint64_t)(cx + 2147483648LL);
}
typedef struct { gent* e; size_t n; double d; } grid_t;

static void grid_build(grid_t* g, const orc_space* s, const uint32_t* slots, size_t n) {
    g->d = s->d; g->n = n;
    g->e = (gent*)malloc((n ? n : 1) * sizeof(gent));
    for (size_t i = 0; i < n; ++i) {
        uint32_t b = slots[i];
        g->e[i].key = cell_key(cell_of(s->ac[0][b], g->d), cell_of(s->ac[1][b], g->d));
        g->e[i].slot = b;
    }
    sort_n(g->e, n, sizeof(gent), cmp_gent);
}
static size_t lower_key(const grid_t* g, uint64_t k) {
    size_t lo = 0, hi = g->n;
    while (lo < hi) { size_t m = (lo + hi) / 2; if (g->e[m].key < k) lo = m + 1; else hi = m; }
    return lo;
}
/* visit every grid entity whose cell intersects A's conservatively widened
 * window: [x-d-m, x+d+m] with m covering float32 rounding of fl(b+-d), so every
 * b with inWin_A(b) OR inWin_b(A) is visited. */
typedef void (*visit_fn)(void* ctx, uint32_t b);
static void grid_query(const grid_t* g, float x, float z, visit_fn fn, void* ctx) {
    double d = g->d;
    double mx = (fabs((double)x) + d) * 9.5367431640625e-07 + 1e-30;   /* 2^-20 */
    double mz = (fabs((double)z) + d) * 9.5367431640625e-07 + 1e-30;
    int64_t cx0 = cell_of((double)x - d - mx, d), cx1 = cell_of((double)x + d + mx, d);
    int64_t cz0 = cell_of((double)z - d - mz, d), cz1 = cell_of((double)z + d + mz, d);
    for (int64_t cz = cz0; cz <= cz1; ++cz) {
        size_t p = lower_key(g, cell_key(cx0, cz));
        uint64_t kend = cell_key(cx1, cz);
        for (; p < g->n && g->e[p].key <= kend; ++p) fn(ctx, g->e[p].slot);
    }
}

/* ------------------------------------------------------------------------ */
/* bulk build == sequential Enter in index order, relations only             */
typedef struct { orc_space* s; uint32_t a; const int32_t* ord; } bulk_ctx;
static void bulk_visit(void* vc, uint32_t b) {
    bulk_ctx* c = (bulk_ctx*)vc;
    orc_space* s = c->s;
    if (b == c->a || c->ord[b] >= c->ord[c->a]) return;  /* pair decided by later-entered */
    if (!orc_in_window(s->ac[0][c->a], s->ac[1][c->a], s->d, s->ac[0][b], s->ac[1][b])) return;
    v_push(&s->nb[c->a], b); v_push(&s->nb[b], c->a);
    if (s->in) {
        v_push(&s->in[c->a], b); v_push(&s->by[b], c->a);
        v_push(&s->in[b], c->a); v_push(&s->by[c->a], b);
    }
}
typedef struct { float c; int32_t ord; int32_t slot; } lent;
static int cmp_lent(const void* a, const void* b) {
    const lent* x = (const lent*)a; const lent* y = (const lent*)b;
    if (x->c != y->c) return x->c < y->c ? -1 : 1;
    return y->ord - x->ord;            /* later insert goes before equal coords */
}

int orc_bulk_enter(orc_space* s, uint32_t n, const uint32_t* slots,
                   const float* x, const float* y, const float* z, const float* yaw,
                   uint8_t sync_flags) {
    for (uint32_t i = 0; i < s->cap; ++i) if (s->present[i]) return GW_ESTATE;  /* empty space only */
    int32_t* ord = (int32_t*)malloc((size_t)s->cap * 4);
    for (uint32_t i = 0; i < s->cap; ++i) ord[i] = -1;
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t a = slots[i];
        if (a >= s->cap || ord[a] >= 0) { free(ord); return GW_EINVAL; }
        ord[a] = (int32_t)i;
        s->present[a] = 1;
        s->ac[0][a] = x[i]; s->ac[1][a] = z[i];
        s->px[a] = x[i]; s->py[a] = y[i]; s->pz[a] = z[i]; s->pyaw[a] = yaw[i];
        s->flags[a] |= sync_flags;                     /* Space.go:196 */
    }
    grid_t g; grid_build(&g, s, slots, n);
    bulk_ctx c = { s, 0, ord };
    for (uint32_t i = 0; i < n; ++i) { c.a = slots[i]; grid_query(&g, x[i], z[i], bulk_visit, &c); }
    free(g.e);
    if (s->mode == ORC_XZLIST) {
        lent* L = (lent*)malloc((size_t)(n ? n : 1) * sizeof(lent));
        for (int ax = 0; ax < 2; ++ax) {
            for (uint32_t i = 0; i < n; ++i) { L[i].c = s->ac[ax][slots[i]]; L[i].ord = (int32_t)i; L[i].slot = (int32_t)slots[i]; }
            sort_n(L, n, sizeof(lent), cmp_lent);
            for (uint32_t i = 0; i < n; ++i) {
                int32_t a = L[i].slot;
                s->node[a].prev[ax] = i ? L[i - 1].slot : -1;
                s->node[a].next[ax] = (i + 1 < n) ? L[i + 1].slot : -1;
                s->node[a].mark = 0;
            }
            s->head[ax] = n ? L[0].slot : -1;
            s->tail[ax] = n ? L[n - 1].slot : -1;
        }
        free(L);
    }
    free(ord);
    return 0;
}

/* ------------------------------------------------------------------------ */
/* SEQRULE batched tick                                                      */
typedef struct { orc_space* s; uint32_t a; vec32* out; } sq_ctx;
static int rel_seq(const orc_space* s, uint32_t a, uint32_t b) {
    /* pair decided by the member with the larger last-op seq (non-movers -1) */
    uint32_t c = s->seq[a] > s->seq[b] ? a : b, o = c == a ? b : a;
    return orc_in_window(s->ac[0][c], s->ac[1][c], s->d, s->ac[0][o], s->ac[1][o]);
}
static void sq_visit(void* vc, uint32_t b) {
    sq_ctx* c = (sq_ctx*)vc;
    if (b == c->a) return;
    if (rel_seq(c->s, c->a, b)) v_push(c->out, b);
}

static void push_ev(gw_event** arr, uint64_t* n, uint64_t* cap, uint32_t w, uint32_t t) {
    if (*n == *cap) { *cap = *cap ? *cap * 2 : 1024; *arr = (gw_event*)realloc(*arr, *cap * sizeof(gw_event)); }
    (*arr)[*n].watcher = w; (*arr)[*n].target = t; (*n)++;
}
static int cmp_ev(const void* a, const void* b) {
    const gw_event* x = (const gw_event*)a; const gw_event* y = (const gw_event*)b;
    if (x->watcher != y->watcher) return x->watcher < y->watcher ? -1 : 1;
    return x->target < y->target ? -1 : x->target > y->target;
}

static void seqrule_relations(orc_space* s, const uint32_t* touched, uint32_t nt) {
    uint32_t* movers = (uint32_t*)malloc((size_t)(nt ? nt : 1) * 4);
    uint32_t nm = 0;
    for (uint32_t i = 0; i < nt; ++i) if (s->seq[touched[i]] >= 0) movers[nm++] = touched[i];
    /* grid over all present entities at final positions */
    uint32_t* pres = (uint32_t*)malloc((size_t)s->cap * 4);
    uint32_t np = 0;
    for (uint32_t i = 0; i < s->cap; ++i) if (s->present[i]) pres[np++] = i;
    grid_t g; grid_build(&g, s, pres, np);
    vec32* nw = (vec32*)calloc(s->cap, sizeof(vec32));       /* new lists of affected slots */
    uint8_t* aff = s->mk;                                     /* affected flag */
    uint32_t* afflist = (uint32_t*)malloc((size_t)s->cap * 4);
    uint32_t naff = 0;
    for (uint32_t i = 0; i < nm; ++i) {
        uint32_t a = movers[i];
        if (!aff[a]) { aff[a] = 1; afflist[naff++] = a; }
        if (s->present[a]) {
            sq_ctx c = { s, a, &nw[a] };
            grid_query(&g, s->ac[0][a], s->ac[1][a], sq_visit, &c);
        }
    }
    /* non-movers: keep non-mover neighbours, add movers that now relate */
    for (uint32_t i = 0; i < nm; ++i) {
        uint32_t a = movers[i];
        for (uint32_t j = 0; j < s->nb[a].n; ++j) {           /* old neighbours of movers */
            uint32_t b = s->nb[a].a[j];
            if (s->seq[b] < 0 && !aff[b]) { aff[b] = 1; afflist[naff++] = b; }
        }
        for (uint32_t j = 0; j < nw[a].n; ++j) {
            uint32_t b = nw[a].a[j];
            if (s->seq[b] < 0) {
                if (!aff[b]) { aff[b] = 1; afflist[naff++] = b; }
                v_push(&nw[b], a);
            }
        }
    }
    for (uint32_t i = 0; i < naff; ++i) {
        uint32_t b = afflist[i];
        if (s->seq[b] >= 0) continue;
        for (uint32_t j = 0; j < s->nb[b].n; ++j) {
            uint32_t c = s->nb[b].a[j];
            if (s->seq[c] < 0) v_push(&nw[b], c);
        }
    }
    /* diff old vs new per affected slot */
    uint64_t cape = 0, capl = 0;
    for (uint32_t i = 0; i < naff; ++i) {
        uint32_t b = afflist[i];
        vec32* o = &s->nb[b]; vec32* n = &nw[b];
        sort_n(o->a, o->n, 4, cmp_u32);
        sort_n(n->a, n->n, 4, cmp_u32);
        uint32_t p = 0, q = 0;
        while (p < o->n || q < n->n) {
            if (q >= n->n || (p < o->n && o->a[p] < n->a[q])) { push_ev(&s->leave, &s->n_leave, &capl, b, o->a[p]); ++p; }
            else if (p >= o->n || n->a[q] < o->a[p]) { push_ev(&s->enter, &s->n_enter, &cape, b, n->a[q]); ++q; }
            else { ++p; ++q; }
        }
    }
    for (uint32_t i = 0; i < naff; ++i) {
        uint32_t b = afflist[i];
        vec32 t = s->nb[b]; s->nb[b] = nw[b]; nw[b] = t;
        aff[b] = 0;
    }
    for (uint32_t i = 0; i < s->cap; ++i) v_free(&nw[i]);
    free(nw); free(afflist); free(g.e); free(pres); free(movers);
    sort_n(s->enter, s->n_enter, sizeof(gw_event), cmp_ev);
    sort_n(s->leave, s->n_leave, sizeof(gw_event), cmp_ev);
}

/* raw stream -> net events by cancellation */
static int cmp_raw(const void* a, const void* b) {
    const rawev* x = (const rawev*)a; const rawev* y = (const rawev*)b;
    return x->key < y->key ? -1 : x->key > y->key;
}
static int net_from_raw(orc_space* s) {
    sort_n(s->raw, s->nraw, sizeof(rawev), cmp_raw);
    uint64_t cape = 0, capl = 0;
    for (size_t i = 0; i < s->nraw;) {
        size_t j = i; int sum = 0;
        while (j < s->nraw && s->raw[j].key == s->raw[i].key) sum += s->raw[j++].d;
        uint32_t w = (uint32_t)(s->raw[i].key >> 32), t = (uint32_t)s->raw[i].key;
        if (sum == 1) push_ev(&s->enter, &s->n_enter, &cape, w, t);
        else if (sum == -1) push_ev(&s->leave, &s->n_leave, &capl, w, t);
        else if (sum != 0) return GW_ESTATE;     /* enter/leave must alternate */
        i = j;
    }
    return 0;
}

int orc_tick(orc_space* s, const gw_op* ops, uint32_t n) {
    s->nraw = 0; s->raw_enter = s->raw_leave = s->create_msgs = s->destroy_msgs = 0;
    s->n_enter = s->n_leave = 0;
    uint32_t* touched = (uint32_t*)malloc((size_t)(n ? n : 1) * 4);
    uint32_t nt = 0;
    int rc = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const gw_op* op = &ops[i];
        uint32_t a = op->slot;
        if (a >= s->cap) { rc = GW_ERANGE; break; }
        switch (op->kind) {
        case GW_OP_ENTER:
            if (s->present[a]) { rc = GW_ESTATE; break; }
            s->present[a] = 1;
            s->ac[0][a] = op->x; s->ac[1][a] = op->z;
            break;
        case GW_OP_MOVED:
            if (!s->present[a]) { rc = GW_ESTATE; break; }
            break;
        case GW_OP_LEAVE:
        case GW_OP_SYNC:
            if (!s->present[a]) { rc = GW_ESTATE; break; }
            break;
        default: rc = GW_EINVAL;
        }
        if (rc) break;
        /* sync state and syncInfoFlag, in call order */
        /* Space.leave leaves syncInfoFlag alone (Space.go:219-242): a Leave's
         * sync_flags is the mask of pending bits the entity keeps (3 = all: it
         * stays in the game in the nil space; 0: destroyed / entering another
         * AOI space, whose Enter flags it anew) */
        if (op->kind == GW_OP_LEAVE) { s->flags[a] &= op->sync_flags; }
        else {
            s->flags[a] |= op->sync_flags;
            s->px[a] = op->x; s->py[a] = op->y; s->pz[a] = op->z; s->pyaw[a] = op->yaw;
        }
        if (op->kind == GW_OP_SYNC) continue;
        if (s->mode == ORC_SEQRULE) {
            if (s->seq[a] < 0 && !s->mk2[a]) { s->mk2[a] = 1; touched[nt++] = a; }
            s->seq[a] = (int32_t)i;
            if (op->kind == GW_OP_MOVED) { s->ac[0][a] = op->x; s->ac[1][a] = op->z; }
            if (op->kind == GW_OP_LEAVE) s->present[a] = 0;
        } else if (s->mode == ORC_XZLIST) {
            if (op->kind == GW_OP_ENTER) xz_enter(s, (int32_t)a);
            else if (op->kind == GW_OP_MOVED) {
                float ox = s->ac[0][a], oz = s->ac[1][a];
                s->ac[0][a] = op->x; s->ac[1][a] = op->z;
                xz_moved(s, (int32_t)a, ox, oz);
            } else { s->present[a] = 0; xz_leave(s, (int32_t)a); }
        } else {  /* BRUTE */
            if (op->kind == GW_OP_MOVED) { s->ac[0][a] = op->x; s->ac[1][a] = op->z; }
            if (op->kind == GW_OP_LEAVE) s->present[a] = 0;
            brute_adjust(s, (int32_t)a);
        }
    }
    if (s->mode == ORC_SEQRULE) {
        if (!rc) seqrule_relations(s, touched, nt);
        for (uint32_t i = 0; i < nt; ++i) { s->seq[touched[i]] = -1; s->mk2[touched[i]] = 0; }
    } else if (!rc) {
        rc = net_from_raw(s);
    }
    free(touched);
    return rc;
}

void orc_event_counts(const orc_space* s, uint64_t* ne, uint64_t* nl) { *ne = s->n_enter; *nl = s->n_leave; }
void orc_events_copy(const orc_space* s, gw_event* e, gw_event* l) {
    if (e && s->n_enter) memcpy(e, s->enter, s->n_enter * sizeof(gw_event));
    if (l && s->n_leave) memcpy(l, s->leave, s->n_leave * sizeof(gw_event));
}
void orc_raw_counts(const orc_space* s, uint64_t* re, uint64_t* rl, uint64_t* cm, uint64_t* dm) {
    *re = s->raw_enter; *rl = s->raw_leave; *cm = s->create_msgs; *dm = s->destroy_msgs;
}

void orc_set_client(orc_space* s, uint32_t slot, uint16_t gate) { if (slot < s->cap) s->gate[slot] = gate; }

/* ------------------------------------------------------------------------ */
/* CollectEntitySyncInfos (Entity.go:1221-1267)                              */
static const uint16_t* g_sort_gate;   /* comparator context (single-threaded oracle) */
static int cmp_rec(const void* a, const void* b) {
    const gw_sync_record* x = (const gw_sync_record*)a; const gw_sync_record* y = (const gw_sync_record*)b;
    uint16_t gx = g_sort_gate[x->watcher], gy = g_sort_gate[y->watcher];
    if (gx != gy) return gx < gy ? -1 : 1;
    if (x->entity != y->entity) return x->entity < y->entity ? -1 : 1;
    return x->watcher < y->watcher ? -1 : x->watcher > y->watcher;
}
static void push_rec(orc_space* s, uint64_t* cap, uint32_t w, uint32_t e) {
    if (s->n_rec == *cap) { *cap = *cap ? *cap * 2 : 1024; s->rec = (gw_sync_record*)realloc(s->rec, *cap * sizeof(gw_sync_record)); }
    gw_sync_record* r = &s->rec[s->n_rec++];
    r->watcher = w; r->entity = e;
    r->x = s->px[e]; r->y = s->py[e]; r->z = s->pz[e]; r->yaw = s->pyaw[e];   /* getSyncInfo, Entity.go:1269-1276 */
}
uint64_t orc_collect(orc_space* s) {
    s->n_rec = 0;
    uint64_t cap = 0;
    for (uint32_t e = 0; e < s->cap; ++e) {
        uint8_t f = s->flags[e];
        if (!f) continue;
        s->flags[e] = 0;
        /* every entity of the game is scanned (Entity.go:1221-1239): one that
         * left into the nil space still syncs its own client; it has no
         * InterestedBy left */
        if ((f & GW_SIF_OWN_CLIENT) && s->gate[e]) push_rec(s, &cap, e, e);
        if (!s->present[e]) continue;
        if (f & GW_SIF_NEIGHBOR_CLIENTS) {
            const vec32* by = s->by ? &s->by[e] : &s->nb[e];        /* e.InterestedBy */
            for (uint32_t j = 0; j < by->n; ++j)
                if (s->gate[by->a[j]]) push_rec(s, &cap, by->a[j], e);
        }
    }
    g_sort_gate = s->gate;
    sort_n(s->rec, s->n_rec, sizeof(gw_sync_record), cmp_rec);
    return s->n_rec;
}
void orc_records_copy(const orc_space* s, gw_sync_record* out) {
    if (s->n_rec) memcpy(out, s->rec, s->n_rec * sizeof(gw_sync_record));
}

/* uuid.go:15-24,48-59: base64 (alphabet A-Z a-z 0-9 _ .), no padding, of 12
 * bytes; GenFixedUUID left-pads shorter input with zeros. */
void orc_fixed_uuid_u32(uint32_t v, char out[16]) {
    static const char* A = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789_.";
    uint8_t b[12] = {0};
    b[8] = (uint8_t)(v >> 24); b[9] = (uint8_t)(v >> 16); b[10] = (uint8_t)(v >> 8); b[11] = (uint8_t)v;
    for (int i = 0, o = 0; i < 12; i += 3, o += 4) {
        out[o] = A[b[i] >> 2];
        out[o + 1] = A[((b[i] & 3) << 4) | (b[i + 1] >> 4)];
        out[o + 2] = A[((b[i + 1] & 15) << 2) | (b[i + 2] >> 6)];
        out[o + 3] = A[b[i + 2] & 63];
    }
}
static uint8_t* put_u16(uint8_t* p, uint16_t v) { p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); return p + 2; }
static uint8_t* put_f32(uint8_t* p, float f) { uint32_t u; memcpy(&u, &f, 4); p[0] = (uint8_t)u; p[1] = (uint8_t)(u >> 8); p[2] = (uint8_t)(u >> 16); p[3] = (uint8_t)(u >> 24); return p + 4; }

uint64_t orc_encode_wire(const orc_space* s, uint8_t* out) {
    uint64_t bytes = 0;
    uint8_t* p = out;
    for (uint64_t i = 0; i < s->n_rec;) {
        uint16_t g = s->gate[s->rec[i].watcher];
        uint64_t j = i;
        while (j < s->n_rec && s->gate[s->rec[j].watcher] == g) ++j;
        bytes += 4 + 48 * (j - i);
        if (out) {
            p = put_u16(p, 1502);                    /* MT_SYNC_POSITION_YAW_ON_CLIENTS, proto.go:107-109 */
            p = put_u16(p, g);                       /* gateid, Entity.go:1216 */
            for (uint64_t k = i; k < j; ++k) {
                const gw_sync_record* r = &s->rec[k];
                orc_fixed_uuid_u32(r->watcher | 0x80000000u, (char*)p); p += 16;  /* AppendClientID */
                orc_fixed_uuid_u32(r->entity, (char*)p); p += 16;                  /* AppendEntityID */
                p = put_f32(p, r->x); p = put_f32(p, r->y); p = put_f32(p, r->z); p = put_f32(p, r->yaw);
            }
        }
        i = j;
    }
    return bytes;
}

static uint32_t copy_sorted(const vec32* v, uint32_t* buf, uint32_t cap) {
    uint32_t* tmp = (uint32_t*)malloc((size_t)(v->n ? v->n : 1) * 4);
    if (v->n) memcpy(tmp, v->a, (size_t)v->n * 4);
    sort_n(tmp, v->n, 4, cmp_u32);
    uint32_t k = v->n < cap ? v->n : cap;
    if (buf && k) memcpy(buf, tmp, (size_t)k * 4);
    free(tmp);
    return v->n;
}
uint32_t orc_neighbors(const orc_space* s, uint32_t slot, uint32_t* buf, uint32_t cap) {
    if (slot >= s->cap) return 0;
    return copy_sorted(s->in ? &s->in[slot] : &s->nb[slot], buf, cap);
}
uint32_t orc_interested_by(const orc_space* s, uint32_t slot, uint32_t* buf, uint32_t cap) {
    if (slot >= s->cap) return 0;
    return copy_sorted(s->by ? &s->by[slot] : &s->nb[slot], buf, cap);
}
uint64_t orc_total_neighbors(const orc_space* s) {
    uint64_t t = 0;
    for (uint32_t i = 0; i < s->cap; ++i) t += s->in ? s->in[i].n : s->nb[i].n;
    return t;
}
int orc_present(const orc_space* s, uint32_t slot) { return slot < s->cap ? s->present[slot] : 0; }

/* keep cmp_u64 referenced for future digest helpers */
int orc__unused_cmp_u64(const void* a, const void* b) { return cmp_u64(a, b); }

/* ------------------------------------------------------------------------ */
/* Client messages, restated on the oracle's state.  */
/* Order of every stream: (gate(watcher), watcher, ...), i.e. one run per     */
/* client inside a gate; the reference sends them from Go map iteration, so  */
/* only the per-client order is meaningful, and that is call order.          */
static const orc_space* g_fs;    /* qsort context (single-threaded oracle) */
static int cmp_gate_rec3(const void* a, const void* b) {
    const uint32_t* x = (const uint32_t*)a; const uint32_t* y = (const uint32_t*)b;
    uint32_t gx = g_fs->gate[x[0]], gy = g_fs->gate[y[0]];
    if (gx != gy) return gx < gy ? -1 : 1;
    if (x[0] != y[0]) return x[0] < y[0] ? -1 : 1;
    if (x[2] != y[2]) return x[2] < y[2] ? -1 : 1;
    return 0;
}
/* Entity.interest / uninterest (Entity.go:236-246) -> e.client.sendCreateEntity
 * (other, false) with other's Position and yaw (GameClient.go:37-53) /
 * sendDestroyEntity(other) (GameClient.go:55-59); a nil client sends nothing.
 * Built from the tick's net events (already in (watcher, target) order), kept
 * stable per gate by a counting pass over the gate ids.  out NULL: count. */
static uint64_t client_msgs(const orc_space* s, const gw_event* ev, uint64_t n, gw_sync_record* cr, gw_event* de) {
    uint64_t* at = (uint64_t*)calloc(65537, 8);
    for (uint64_t i = 0; i < n; ++i) at[s->gate[ev[i].watcher] + 1]++;
    at[1] = 0;                                   /* gate 0: no client, no message */
    for (uint32_t g = 1; g <= 65535u; ++g) at[g + 1] += at[g];
    const uint64_t k = at[65536];
    if (cr || de) {
        for (uint64_t i = 0; i < n; ++i) {       /* stable: events stay in (watcher, target) order */
            uint32_t w = ev[i].watcher, t = ev[i].target, g = s->gate[w];
            if (!g) continue;
            uint64_t j = at[g]++;
            if (cr) {
                gw_sync_record r = {w, t, s->px[t], s->py[t], s->pz[t], s->pyaw[t]};
                cr[j] = r;
            } else {
                de[j] = ev[i];
            }
        }
    }
    free(at);
    return k;
}
uint64_t orc_client_creates(const orc_space* s, gw_sync_record* out) {
    return client_msgs(s, s->enter, s->n_enter, out, NULL);
}
uint64_t orc_client_destroys(const orc_space* s, gw_event* out) {
    return client_msgs(s, s->leave, s->n_leave, NULL, out);
}
/* Entity.CallAllClients (Entity.go:743-749) and the AllClients attribute
 * notifications (Entity.go:814-917): e.client.call(...), then for neighbor in
 * e.InterestedBy: neighbor.client.call(...).  Call k on slots[k] yields
 * {watcher, entity, k} records (3 words); out NULL: count. */
uint64_t orc_fanout(const orc_space* s, const uint32_t* slots, uint32_t n, uint32_t* out) {
    uint64_t k = 0;
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t e = slots[i];
        if (e >= s->cap) continue;
        if (s->gate[e]) {
            if (out) { out[3 * k] = e; out[3 * k + 1] = e; out[3 * k + 2] = i; }
            ++k;
        }
        const vec32* by = s->by ? &s->by[e] : &s->nb[e];
        for (uint32_t j = 0; j < by->n; ++j) {
            uint32_t w = by->a[j];
            if (!s->gate[w]) continue;
            if (out) { out[3 * k] = w; out[3 * k + 1] = e; out[3 * k + 2] = i; }
            ++k;
        }
    }
    if (out && k) {
        g_fs = s;
        sort_n(out, k, 12, cmp_gate_rec3);
    }
    return k;
}
