/*
 * orc_replay.c — TEST INFRASTRUCTURE ONLY: a standalone driver of the CPU
 * oracle (orc.c), built with AddressSanitizer + UndefinedBehaviorSanitizer by
 * `make -C oracle san` (sanitizers on the CPU restatement).
 * It replays a trace file through one oracle engine exactly as
 * tests/test_golden.py does through ctypes (bulk Enter with pending flags 3,
 * clients, then per tick: orc_tick, events, orc_collect, the wire encoding,
 * client messages and a fan-out), so the sanitizers see every path the golden
 * fixtures exercise; tests/test_oracle_sanitized.py compares the output with
 * the fixtures.
 *
 * usage: orc_replay MODE IN OUT      (MODE 0 XZList, 1 brute force, 2 seq rule)
 *   IN: the c_harness trace format (tests/c_harness.c): "GWH1", u32 capacity,
 *       f32 d, f32 bounds[4], u32 n_init, u32 n_ticks; n_init x {u32 slot, f32
 *       x, y, z, yaw}; capacity x u16 gate; per tick u32 n_ops + gw_op[n_ops]
 *   OUT per tick: u64 n_enter + enters, u64 n_leave + leaves, u64 n_rec +
 *       records (24 B), u64 wire bytes + bytes, u64 creates, u64 destroys,
 *       u64 fan-out deliveries; then u64 total neighbours and, per slot,
 *       u32 count + the InterestedIn list.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "orc.h"

static void rd(void* p, size_t n, FILE* f) {
    if (n && fread(p, 1, n, f) != n) {
        fprintf(stderr, "orc_replay: short input\n");
        exit(2);
    }
}

static void wr(const void* p, size_t n, FILE* f) {
    if (n && fwrite(p, 1, n, f) != n) {
        fprintf(stderr, "orc_replay: short write\n");
        exit(2);
    }
}

static void* xmalloc(size_t n) {
    void* p = malloc(n ? n : 1);
    if (!p) {
        fprintf(stderr, "orc_replay: out of memory\n");
        exit(2);
    }
    return p;
}

static void wr_u64(uint64_t v, FILE* f) { wr(&v, 8, f); }

int main(int argc, char** argv) {
    if (argc != 4) {
        fprintf(stderr, "usage: orc_replay MODE IN OUT\n");
        return 2;
    }
    const int mode = atoi(argv[1]);
    FILE* in = fopen(argv[2], "rb");
    FILE* out = fopen(argv[3], "wb");
    if (!in || !out || mode < ORC_XZLIST || mode > ORC_SEQRULE) {
        fprintf(stderr, "orc_replay: bad arguments\n");
        return 2;
    }
    char magic[4];
    uint32_t cap, n_init, n_ticks;
    float d, bounds[4];
    rd(magic, 4, in);
    if (memcmp(magic, "GWH1", 4)) {
        fprintf(stderr, "orc_replay: bad magic\n");
        return 2;
    }
    rd(&cap, 4, in);
    rd(&d, 4, in);
    rd(bounds, 16, in);
    rd(&n_init, 4, in);
    rd(&n_ticks, 4, in);
    uint32_t* slots = xmalloc((size_t)n_init * 4);
    float *x = xmalloc((size_t)n_init * 4), *y = xmalloc((size_t)n_init * 4), *z = xmalloc((size_t)n_init * 4),
          *yaw = xmalloc((size_t)n_init * 4);
    for (uint32_t i = 0; i < n_init; ++i) {
        rd(&slots[i], 4, in);
        rd(&x[i], 4, in);
        rd(&y[i], 4, in);
        rd(&z[i], 4, in);
        rd(&yaw[i], 4, in);
    }
    uint16_t* gates = xmalloc((size_t)cap * 2);
    rd(gates, (size_t)cap * 2, in);

    orc_space* s = orc_new(cap, d, mode);
    if (!s || orc_bulk_enter(s, n_init, slots, x, y, z, yaw, 3)) {
        fprintf(stderr, "orc_replay: load failed\n");
        return 2;
    }
    for (uint32_t i = 0; i < cap; ++i)
        if (gates[i]) orc_set_client(s, i, gates[i]);
    uint32_t* calls = xmalloc((size_t)cap * 4);
    for (uint32_t t = 0; t < n_ticks; ++t) {
        uint32_t n;
        rd(&n, 4, in);
        gw_op* ops = xmalloc((size_t)n * sizeof(gw_op));
        rd(ops, (size_t)n * sizeof(gw_op), in);
        if (orc_tick(s, ops, n)) {
            fprintf(stderr, "orc_replay: tick %u rejected\n", t);
            return 2;
        }
        uint64_t ne, nl;
        orc_event_counts(s, &ne, &nl);
        gw_event* e = xmalloc(ne * sizeof(gw_event));
        gw_event* l = xmalloc(nl * sizeof(gw_event));
        orc_events_copy(s, e, l);
        wr_u64(ne, out);
        wr(e, ne * sizeof(gw_event), out);
        wr_u64(nl, out);
        wr(l, nl * sizeof(gw_event), out);
        // client messages of the tick's events and a fan-out of one call per op
        const uint64_t ncr = orc_client_creates(s, NULL), nde = orc_client_destroys(s, NULL);
        gw_sync_record* cr = xmalloc(ncr * sizeof(gw_sync_record));
        gw_event* de = xmalloc(nde * sizeof(gw_event));
        orc_client_creates(s, cr);
        orc_client_destroys(s, de);
        uint32_t nc = 0;
        for (uint32_t i = 0; i < n && nc < cap; ++i)
            if (orc_present(s, ops[i].slot)) calls[nc++] = ops[i].slot;
        const uint64_t nfo = orc_fanout(s, calls, nc, NULL);
        uint32_t* fo = xmalloc(nfo * 12);
        orc_fanout(s, calls, nc, fo);
        const uint64_t nr = orc_collect(s);
        gw_sync_record* r = xmalloc(nr * sizeof(gw_sync_record));
        orc_records_copy(s, r);
        wr_u64(nr, out);
        wr(r, nr * sizeof(gw_sync_record), out);
        const uint64_t nw = orc_encode_wire(s, NULL);
        uint8_t* w = xmalloc(nw);
        if (orc_encode_wire(s, w) != nw) {
            fprintf(stderr, "orc_replay: wire length changed\n");
            return 2;
        }
        wr_u64(nw, out);
        wr(w, nw, out);
        wr_u64(ncr, out);
        wr_u64(nde, out);
        wr_u64(nfo, out);
        free(w);
        free(r);
        free(fo);
        free(de);
        free(cr);
        free(l);
        free(e);
        free(ops);
    }
    wr_u64(orc_total_neighbors(s), out);
    uint32_t* nb = xmalloc((size_t)cap * 4);
    for (uint32_t i = 0; i < cap; ++i) {
        const uint32_t k = orc_neighbors(s, i, nb, cap);
        wr(&k, 4, out);
        wr(nb, (size_t)k * 4, out);
    }
    free(nb);
    free(calls);
    orc_free(s);
    free(gates);
    free(yaw);
    free(z);
    free(y);
    free(x);
    free(slots);
    if (fclose(out)) return 2;
    fclose(in);
    return 0;
}
