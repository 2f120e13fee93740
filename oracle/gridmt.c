/*
 * gridmt.c — multi-threaded uniform-grid CPU implementation of one AOI tick
 * and one sync collect under the batched contract (orc.h ORC_SEQRULE), for
 * the fairness point SURVEY.md 8(d) asks next to the single-thread XZList
 * baseline: "a multi-threaded uniform-grid CPU implementation on all host
 * cores, stating the core count".
 *
 * BENCH / TEST INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg and
 * tests/test_oracle.py); nothing in goworld_amd/ uses it.  Checked against
 * orc.c's SEQRULE engine event for event and record for record.
 *
 * Per entity: AOI position, presence, the global stamp of its last AOI op.
 * The relation of a pair is decided by the member with the larger stamp (its
 * rounded window must hold the other; orc.c rel_seq).  A tick:
 *   1. ops in call order (sequential, O(M)): flags / payload, last AOI op per
 *      slot; movers keep their pre-tick position, presence and stamp;
 *   2. cell lists of all present entities (cells of side d), rebuilt by a
 *      parallel counting sort, and cell lists of the movers' old positions;
 *   3. per mover, in parallel: its old and new neighbour sets from the cells
 *      around its old and new windows, sorted and diffed -> own events, and
 *      the mirror events of op-less neighbours;
 *   4. enter / leave arrays sorted by (watcher, target) with a parallel LSD
 *      radix sort.
 * The collect walks each flagged entity's window (parallel) and writes its
 * records at scanned offsets, entities in slot order.
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/gpuaoi.h"

typedef struct {
    uint32_t cap, W, H, nthreads;
    float d, x0, z0, cs;
    float *x, *z;                    /* AOI position (Position.X, Position.Z) */
    uint8_t* present;
    uint64_t* stamp;                 /* global stamp of the last AOI op */
    float *px, *py, *pz, *pyaw;      /* sync payload */
    uint32_t* flags;
    uint16_t* gate;
    uint64_t next_stamp;
    /* per tick */
    int32_t* last_aoi;               /* [cap] op index or -1 */
    uint32_t *cell_start, *cell_ent; /* present entities by cell (new positions) */
    uint32_t *ocell_start, *ocell_ent; /* movers by cell of their old position */
    uint64_t *enter, *leave;         /* watcher << 32 | target */
    uint64_t n_enter, n_leave;
    gw_sync_record* rec;
    uint64_t n_rec;
} gmt;

static int cell_x(const gmt* g, float x) {
    float f = floorf((x - g->x0) / g->cs);
    return f < 0 ? 0 : (f >= (float)g->W ? (int)g->W - 1 : (int)f);
}
static int cell_z(const gmt* g, float z) {
    float f = floorf((z - g->z0) / g->cs);
    return f < 0 ? 0 : (f >= (float)g->H ? (int)g->H - 1 : (int)f);
}
static int in_win(float cx, float cz, float d, float ox, float oz) {
    return ox >= cx - d && ox <= cx + d && oz >= cz - d && oz <= cz + d;
}
static int related(float d, float ax, float az, uint64_t sa, float bx, float bz, uint64_t sb) {
    return sa > sb ? in_win(ax, az, d, bx, bz) : in_win(bx, bz, d, ax, az);
}

gmt* gmt_new(uint32_t cap, float d, float minx, float minz, float maxx, float maxz, int nthreads) {
    gmt* g = (gmt*)calloc(1, sizeof(gmt));
    g->cap = cap;
    g->d = d;
    g->cs = d;
    g->x0 = minx;
    g->z0 = minz;
    g->W = (uint32_t)ceilf((maxx - minx) / d) + 1;
    g->H = (uint32_t)ceilf((maxz - minz) / d) + 1;
    g->nthreads = nthreads > 0 ? (uint32_t)nthreads : (uint32_t)omp_get_max_threads();
    g->x = (float*)calloc(cap, 4); g->z = (float*)calloc(cap, 4);
    g->present = (uint8_t*)calloc(cap, 1);
    g->stamp = (uint64_t*)calloc(cap, 8);
    g->px = (float*)calloc(cap, 4); g->py = (float*)calloc(cap, 4);
    g->pz = (float*)calloc(cap, 4); g->pyaw = (float*)calloc(cap, 4);
    g->flags = (uint32_t*)calloc(cap, 4);
    g->gate = (uint16_t*)calloc(cap, 2);
    g->last_aoi = (int32_t*)malloc((size_t)cap * 4);
    for (uint32_t i = 0; i < cap; ++i) g->last_aoi[i] = -1;
    size_t nc = (size_t)g->W * g->H + 1;
    g->cell_start = (uint32_t*)calloc(nc, 4);
    g->cell_ent = (uint32_t*)malloc((size_t)cap * 4 + 4);
    g->ocell_start = (uint32_t*)calloc(nc, 4);
    g->ocell_ent = (uint32_t*)malloc((size_t)cap * 4 + 4);
    g->next_stamp = 1;
    return g;
}

void gmt_free(gmt* g) {
    if (!g) return;
    free(g->x); free(g->z); free(g->present); free(g->stamp); free(g->px); free(g->py); free(g->pz);
    free(g->pyaw); free(g->flags); free(g->gate); free(g->last_aoi); free(g->cell_start); free(g->cell_ent);
    free(g->ocell_start); free(g->ocell_ent); free(g->enter); free(g->leave); free(g->rec);
    free(g);
}

void gmt_set_clients(gmt* g, const uint16_t* gates) { memcpy(g->gate, gates, (size_t)g->cap * 2); }

/* cell lists of `ids` at positions (xs, zs): parallel counting sort */
static void build_cells(gmt* g, const uint32_t* ids, uint32_t n, const float* xs, const float* zs,
                        uint32_t* start, uint32_t* ent) {
    const size_t nc = (size_t)g->W * g->H;
    const int T = (int)g->nthreads;
    uint32_t* cell = (uint32_t*)malloc((size_t)(n ? n : 1) * 4);
    uint32_t* hist = (uint32_t*)calloc((size_t)T * nc, 4);
#pragma omp parallel num_threads(T)
    {
        const int t = omp_get_thread_num();
        uint32_t* h = hist + (size_t)t * nc;
#pragma omp for schedule(static)
        for (uint32_t i = 0; i < n; ++i) {
            const uint32_t e = ids ? ids[i] : i;
            cell[i] = (uint32_t)cell_z(g, zs[e]) * g->W + (uint32_t)cell_x(g, xs[e]);
            h[cell[i]]++;
        }
    }
    /* cell-major, thread-minor prefix: each thread's entries of a cell keep index order */
    uint32_t acc = 0;
    for (size_t c = 0; c < nc; ++c) {
        start[c] = acc;
        for (int t = 0; t < T; ++t) {
            const uint32_t v = hist[(size_t)t * nc + c];
            hist[(size_t)t * nc + c] = acc;
            acc += v;
        }
    }
    start[nc] = acc;
#pragma omp parallel num_threads(T)
    {
        const int t = omp_get_thread_num();
        uint32_t* h = hist + (size_t)t * nc;
#pragma omp for schedule(static)
        for (uint32_t i = 0; i < n; ++i) ent[h[cell[i]]++] = ids ? ids[i] : i;
    }
    free(hist);
    free(cell);
}

/* bulk load (restore path): present, stamps in load order, no events */
int gmt_load(gmt* g, uint32_t n, const uint32_t* slots, const float* x, const float* y, const float* z,
             const float* yaw) {
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t s = slots[i];
        if (s >= g->cap) return GW_ERANGE;
        g->present[s] = 1;
        g->x[s] = x[i]; g->z[s] = z[i];
        g->px[s] = x[i]; g->py[s] = y[i]; g->pz[s] = z[i]; g->pyaw[s] = yaw[i];
        g->stamp[s] = g->next_stamp++;
        g->flags[s] |= GW_SIF_OWN_CLIENT | GW_SIF_NEIGHBOR_CLIENTS;
    }
    /* cell lists of the loaded population (a collect may come before any tick) */
    uint32_t* pres = (uint32_t*)malloc((size_t)g->cap * 4);
    uint32_t np = 0;
    for (uint32_t i = 0; i < g->cap; ++i) if (g->present[i]) pres[np++] = i;
    build_cells(g, pres, np, g->x, g->z, g->cell_start, g->cell_ent);
    free(pres);
    return 0;
}

typedef struct { uint32_t* a; size_t n, cap; } vec;
static void vpush(vec* v, uint32_t x) {
    if (v->n == v->cap) { v->cap = v->cap ? v->cap * 2 : 256; v->a = (uint32_t*)realloc(v->a, v->cap * 4); }
    v->a[v->n++] = x;
}
typedef struct { uint64_t* a; size_t n, cap; } vec64;
static void vpush64(vec64* v, uint64_t x) {
    if (v->n == v->cap) { v->cap = v->cap ? v->cap * 2 : 1024; v->a = (uint64_t*)realloc(v->a, v->cap * 8); }
    v->a[v->n++] = x;
}
static int cmp_u32(const void* a, const void* b) {
    uint32_t x = *(const uint32_t*)a, y = *(const uint32_t*)b;
    return x < y ? -1 : x > y;
}

/* parallel LSD radix sort of 64-bit keys on their low `bits` bits */
static void radix64(uint64_t* a, uint64_t n, int bits, int T) {
    if (n < 2) return;
    enum { R = 11, B = 1 << R };
    uint64_t* tmp = (uint64_t*)malloc(n * 8);
    uint64_t* hist = (uint64_t*)malloc((size_t)T * B * 8);
    uint64_t *src = a, *dst = tmp;
    for (int sh = 0; sh < bits; sh += R) {
#pragma omp parallel num_threads(T)
        {
            const int t = omp_get_thread_num();
            uint64_t* h = hist + (size_t)t * B;
            memset(h, 0, (size_t)B * 8);
            const uint64_t lo = n * t / T, hi = n * (t + 1) / T;
            for (uint64_t i = lo; i < hi; ++i) h[(src[i] >> sh) & (B - 1)]++;
#pragma omp barrier
#pragma omp single
            {
                uint64_t acc = 0;
                for (int b = 0; b < B; ++b)
                    for (int u = 0; u < T; ++u) {
                        const uint64_t v = hist[(size_t)u * B + b];
                        hist[(size_t)u * B + b] = acc;
                        acc += v;
                    }
            }
            for (uint64_t i = lo; i < hi; ++i) dst[h[(src[i] >> sh) & (B - 1)]++] = src[i];
        }
        uint64_t* s = src; src = dst; dst = s;
    }
    if (src != a) memcpy(a, src, n * 8);
    free(hist);
    free(tmp);
}

static int bits_for(uint32_t v) { int b = 1; while (b < 32 && (1ull << b) < v) ++b; return b; }

/* candidates of the cells around [x-d, x+d] x [z-d, z+d] (a margin covers the rounding of c +- d) */
#define FOR_CELLS(g, cx, cz, start, ent, body)                                                        \
    do {                                                                                              \
        const float m_ = 1e-4f * (fabsf(cx) + fabsf(cz) + (g)->d) + 1e-3f;                            \
        const int x0_ = cell_x(g, (cx) - (g)->d - m_), x1_ = cell_x(g, (cx) + (g)->d + m_);             \
        const int z0_ = cell_z(g, (cz) - (g)->d - m_), z1_ = cell_z(g, (cz) + (g)->d + m_);             \
        for (int zz_ = z0_; zz_ <= z1_; ++zz_)                                                        \
            for (uint32_t k_ = (start)[(size_t)zz_ * (g)->W + x0_];                                   \
                 k_ < (start)[(size_t)zz_ * (g)->W + x1_ + 1]; ++k_) {                                \
                const uint32_t b = (ent)[k_];                                                         \
                body                                                                                  \
            }                                                                                         \
    } while (0)

int gmt_tick(gmt* g, const gw_op* ops, uint32_t n) {
    const int T = (int)g->nthreads;
    const float d = g->d;
    /* 1. ops in call order */
    uint32_t* movers = (uint32_t*)malloc((size_t)(n ? n : 1) * 4);
    uint32_t nm = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const gw_op* op = &ops[i];
        if (op->slot >= g->cap || op->kind < GW_OP_ENTER || op->kind > GW_OP_SYNC) { free(movers); return GW_EINVAL; }
        const uint32_t a = op->slot;
        if (op->kind == GW_OP_LEAVE) g->flags[a] &= op->sync_flags;   /* keep-mask (orc.c) */
        else {
            g->flags[a] |= op->sync_flags;
            g->px[a] = op->x; g->py[a] = op->y; g->pz[a] = op->z; g->pyaw[a] = op->yaw;
        }
        if (op->kind == GW_OP_SYNC) continue;
        if (g->last_aoi[a] < 0) movers[nm++] = a;
        g->last_aoi[a] = (int32_t)i;
    }
    float* ox = (float*)malloc((size_t)(nm ? nm : 1) * 4);
    float* oz = (float*)malloc((size_t)(nm ? nm : 1) * 4);
    uint8_t* op_ = (uint8_t*)malloc(nm ? nm : 1);
    uint64_t* os = (uint64_t*)malloc((size_t)(nm ? nm : 1) * 8);
    uint8_t* is_mover = (uint8_t*)calloc(g->cap, 1);
    float* oxs = (float*)malloc((size_t)g->cap * 4);          /* old positions by slot (movers only) */
    float* ozs = (float*)malloc((size_t)g->cap * 4);
    uint32_t* oid = (uint32_t*)malloc((size_t)(nm ? nm : 1) * 4);
    uint32_t noid = 0;
    for (uint32_t k = 0; k < nm; ++k) {
        const uint32_t a = movers[k];
        ox[k] = g->x[a]; oz[k] = g->z[a]; op_[k] = g->present[a]; os[k] = g->stamp[a];
        oxs[a] = g->x[a]; ozs[a] = g->z[a];
        is_mover[a] = 1;
        if (op_[k]) oid[noid++] = a;
        const gw_op* op = &ops[g->last_aoi[a]];
        if (op->kind == GW_OP_LEAVE) g->present[a] = 0;
        else { g->present[a] = 1; g->x[a] = op->x; g->z[a] = op->z; }
        g->stamp[a] = g->next_stamp + (uint64_t)g->last_aoi[a];
        g->last_aoi[a] = -1;
    }
    g->next_stamp += n;
    /* 2. cell lists */
    uint32_t* pres = (uint32_t*)malloc((size_t)g->cap * 4);
    uint32_t np = 0;
    for (uint32_t i = 0; i < g->cap; ++i) if (g->present[i]) pres[np++] = i;
    build_cells(g, pres, np, g->x, g->z, g->cell_start, g->cell_ent);
    build_cells(g, oid, noid, oxs, ozs, g->ocell_start, g->ocell_ent);
    /* old stamps by slot for movers */
    uint64_t* ost = (uint64_t*)malloc((size_t)g->cap * 8);
    for (uint32_t k = 0; k < nm; ++k) ost[movers[k]] = os[k];
    /* 3. per mover */
    vec64* ent = (vec64*)calloc(T, sizeof(vec64));
    vec64* lev = (vec64*)calloc(T, sizeof(vec64));
#pragma omp parallel num_threads(T)
    {
        const int t = omp_get_thread_num();
        vec so = {0}, sn = {0};
#pragma omp for schedule(dynamic, 64)
        for (uint32_t k = 0; k < nm; ++k) {
            const uint32_t a = movers[k];
            so.n = sn.n = 0;
            if (op_[k]) {
                const float ax = ox[k], az = oz[k];
                const uint64_t sa = os[k];
                /* op-less entities: current position == old one */
                FOR_CELLS(g, ax, az, g->cell_start, g->cell_ent, {
                    if (!is_mover[b] && related(d, ax, az, sa, g->x[b], g->z[b], g->stamp[b])) vpush(&so, b);
                });
                FOR_CELLS(g, ax, az, g->ocell_start, g->ocell_ent, {
                    if (b != a && related(d, ax, az, sa, oxs[b], ozs[b], ost[b])) vpush(&so, b);
                });
            }
            if (g->present[a]) {
                const float ax = g->x[a], az = g->z[a];
                const uint64_t sa = g->stamp[a];
                FOR_CELLS(g, ax, az, g->cell_start, g->cell_ent, {
                    if (b != a && related(d, ax, az, sa, g->x[b], g->z[b], g->stamp[b])) vpush(&sn, b);
                });
            }
            qsort(so.a, so.n, 4, cmp_u32);
            qsort(sn.a, sn.n, 4, cmp_u32);
            size_t p = 0, q = 0;
            while (p < so.n || q < sn.n) {
                if (q >= sn.n || (p < so.n && so.a[p] < sn.a[q])) {          /* leave */
                    const uint32_t b = so.a[p++];
                    vpush64(&lev[t], ((uint64_t)a << 32) | b);
                    if (!is_mover[b]) vpush64(&lev[t], ((uint64_t)b << 32) | a);
                } else if (p >= so.n || sn.a[q] < so.a[p]) {                 /* enter */
                    const uint32_t b = sn.a[q++];
                    vpush64(&ent[t], ((uint64_t)a << 32) | b);
                    if (!is_mover[b]) vpush64(&ent[t], ((uint64_t)b << 32) | a);
                } else { ++p; ++q; }
            }
        }
        free(so.a);
        free(sn.a);
    }
    /* 4. canonical arrays */
    uint64_t ne = 0, nl = 0;
    for (int t = 0; t < T; ++t) { ne += ent[t].n; nl += lev[t].n; }
    g->enter = (uint64_t*)realloc(g->enter, (ne ? ne : 1) * 8);
    g->leave = (uint64_t*)realloc(g->leave, (nl ? nl : 1) * 8);
    ne = nl = 0;
    for (int t = 0; t < T; ++t) {
        if (ent[t].n) memcpy(g->enter + ne, ent[t].a, ent[t].n * 8);
        if (lev[t].n) memcpy(g->leave + nl, lev[t].a, lev[t].n * 8);
        ne += ent[t].n; nl += lev[t].n;
        free(ent[t].a); free(lev[t].a);
    }
    const int kb = 32 + bits_for(g->cap);
    radix64(g->enter, ne, kb, T);
    radix64(g->leave, nl, kb, T);
    g->n_enter = ne; g->n_leave = nl;
    free(ent); free(lev); free(movers); free(ox); free(oz); free(op_); free(os); free(is_mover); free(oxs);
    free(ozs); free(oid); free(pres); free(ost);
    return 0;
}

void gmt_event_counts(const gmt* g, uint64_t* ne, uint64_t* nl) { *ne = g->n_enter; *nl = g->n_leave; }
void gmt_events_copy(const gmt* g, gw_event* e, gw_event* l) {
    for (uint64_t i = 0; i < g->n_enter; ++i) { e[i].watcher = (uint32_t)(g->enter[i] >> 32); e[i].target = (uint32_t)g->enter[i]; }
    for (uint64_t i = 0; i < g->n_leave; ++i) { l[i].watcher = (uint32_t)(g->leave[i] >> 32); l[i].target = (uint32_t)g->leave[i]; }
}

/* CollectEntitySyncInfos (Entity.go:1221-1267): flagged entities in slot
 * order; own record, then one per related neighbour with a client */
uint64_t gmt_collect(gmt* g) {
    const int T = (int)g->nthreads;
    const float d = g->d;
    uint32_t* fl = (uint32_t*)malloc((size_t)g->cap * 4);
    uint32_t nf = 0;
    for (uint32_t i = 0; i < g->cap; ++i) if (g->flags[i]) fl[nf++] = i;
    uint64_t* cnt = (uint64_t*)calloc((size_t)nf + 1, 8);
    vec* nb = (vec*)calloc(nf ? nf : 1, sizeof(vec));
#pragma omp parallel for num_threads(T) schedule(dynamic, 64)
    for (uint32_t k = 0; k < nf; ++k) {
        const uint32_t e = fl[k];
        const uint32_t f = g->flags[e];
        uint64_t c = 0;
        if ((f & GW_SIF_OWN_CLIENT) && g->gate[e]) ++c;       /* also after a Leave (orc.c) */
        if (g->present[e]) {
            if (f & GW_SIF_NEIGHBOR_CLIENTS) {
                const float ex = g->x[e], ez = g->z[e];
                const uint64_t se = g->stamp[e];
                FOR_CELLS(g, ex, ez, g->cell_start, g->cell_ent, {
                    if (b != e && g->gate[b] && related(d, ex, ez, se, g->x[b], g->z[b], g->stamp[b]))
                        vpush(&nb[k], b);
                });
                c += nb[k].n;
            }
        }
        cnt[k] = c;
    }
    uint64_t acc = 0;
    for (uint32_t k = 0; k < nf; ++k) { const uint64_t v = cnt[k]; cnt[k] = acc; acc += v; }
    g->rec = (gw_sync_record*)realloc(g->rec, (acc ? acc : 1) * sizeof(gw_sync_record));
#pragma omp parallel for num_threads(T) schedule(dynamic, 64)
    for (uint32_t k = 0; k < nf; ++k) {
        const uint32_t e = fl[k];
        const uint32_t f = g->flags[e];
        uint64_t at = cnt[k];
        gw_sync_record r;
        r.entity = e; r.x = g->px[e]; r.y = g->py[e]; r.z = g->pz[e]; r.yaw = g->pyaw[e];
        if ((f & GW_SIF_OWN_CLIENT) && g->gate[e]) { r.watcher = e; g->rec[at++] = r; }
        for (size_t j = 0; j < nb[k].n; ++j) { r.watcher = nb[k].a[j]; g->rec[at++] = r; }
        free(nb[k].a);
        g->flags[e] = 0;
    }
    g->n_rec = acc;
    free(nb); free(cnt); free(fl);
    return acc;
}

void gmt_records_copy(const gmt* g, gw_sync_record* out) { memcpy(out, g->rec, g->n_rec * sizeof(gw_sync_record)); }
int gmt_threads(const gmt* g) { return (int)g->nthreads; }
