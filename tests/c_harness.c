/*
 * c_harness.c — a plain-C caller of libgpuaoi.so that replays a trace through
 * the C ABI in the order the Go shim makes the calls for one
 * game, with the host boundary rows of the path included:
 *
 *   load      gw_space_create (Space.EnableAOI, Space.go:91-106), entity and
 *             client ids (GenFixedUUID, uuid/uuid.go:48-59), gw_set_clients,
 *             SetClientSyncing, gw_space_restore (restore path, Space.go:209-214)
 *   per tick  client position records (the Moved ops a client sent: sync
 *             flags NEIGHBOR) packed as MT_SYNC_POSITION_YAW_FROM_CLIENT
 *             payloads (eid[16] f32 x y z yaw, GameService.go:395-407) and
 *             decoded by gw_submit_client_sync; every other op through
 *             gw_submit, in the trace's call order; gw_tick (events to the
 *             host); gw_sync_collect + gw_sync_encode_wire (the game->gate
 *             packets, Entity.go:1210-1266)
 *
 * usage: c_harness IN OUT [--server]
 *   --server: every op goes through gw_submit with its own y / yaw payload
 *             (the server-side Space.enter / Space.move / SetYaw path,
 *             Space.go:179-252, Entity.go:1185-1205,1284-1290), none through
 *             the client-record decode
 *   IN  (little-endian): "GWH1", u32 capacity, f32 d, f32 bounds[4], u32 n_init,
 *       u32 n_ticks; n_init x {u32 slot, f32 x, y, z, yaw}; capacity x u16 gate;
 *       per tick u32 n_ops + n_ops x gw_op (24 B)
 *   OUT per tick: u64 n_enter, enters (8 B each), u64 n_leave, leaves,
 *       u64 wire bytes, the wire bytes, u32 packets, per packet {u32 gate,
 *       u64 offset}; then u32 records-applied-by-decode
 * Exit status 0 on success; a failing ABI call prints gw_last_error.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "gpuaoi.h"

static gw_ctx* g;

static void check(int rc, const char* what) {
    if (rc) {
        fprintf(stderr, "c_harness: %s failed (%d): %s\n", what, rc, gw_last_error(g));
        exit(2);
    }
}

static void rd(void* p, size_t n, FILE* f) {
    if (n && fread(p, 1, n, f) != n) {
        fprintf(stderr, "c_harness: short input\n");
        exit(2);
    }
}

/* uuid.go:15-24,48-59: base64 (A-Z a-z 0-9 _ .) of 12 bytes, the value left-padded with zeros */
static void fixed_uuid(uint32_t v, char out[16]) {
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

static int server_only;   /* --server */

static int is_client_move(const gw_op* o) {
    return !server_only && o->kind == GW_OP_MOVED && o->sync_flags == GW_SIF_NEIGHBOR_CLIENTS;
}

int main(int argc, char** argv) {
    if (argc == 4 && !strcmp(argv[3], "--server")) {
        server_only = 1;
    } else if (argc != 3) {
        fprintf(stderr, "usage: c_harness IN OUT [--server]\n");
        return 2;
    }
    FILE* in = fopen(argv[1], "rb");
    FILE* out = fopen(argv[2], "wb");
    if (!in || !out) {
        fprintf(stderr, "c_harness: cannot open files\n");
        return 2;
    }
    char magic[4];
    uint32_t cap, n_init, n_ticks;
    float d, bounds[4];
    rd(magic, 4, in);
    if (memcmp(magic, "GWH1", 4)) {
        fprintf(stderr, "c_harness: bad magic\n");
        return 2;
    }
    rd(&cap, 4, in); rd(&d, 4, in); rd(bounds, 16, in); rd(&n_init, 4, in); rd(&n_ticks, 4, in);
    uint32_t* slots = malloc((size_t)n_init * 4);
    float *x = malloc((size_t)n_init * 4), *y = malloc((size_t)n_init * 4), *z = malloc((size_t)n_init * 4),
          *yaw = malloc((size_t)n_init * 4);
    for (uint32_t i = 0; i < n_init; ++i) {
        rd(&slots[i], 4, in); rd(&x[i], 4, in); rd(&y[i], 4, in); rd(&z[i], 4, in); rd(&yaw[i], 4, in);
    }
    uint16_t* gates = malloc((size_t)cap * 2);
    rd(gates, (size_t)cap * 2, in);

    if (gw_init(0, &g)) {
        fprintf(stderr, "c_harness: gw_init(0) failed (no HIP device?)\n");
        return 2;
    }
    uint32_t sid, base;
    check(gw_space_create(g, d, cap, bounds, &sid, &base), "gw_space_create");
    uint32_t* all = malloc((size_t)cap * 4);
    char* eids = malloc((size_t)cap * 16);
    char* cids = malloc((size_t)cap * 16);
    uint8_t* on = malloc(cap);
    uint32_t nc = 0;
    uint32_t* cs = malloc((size_t)cap * 4);
    uint16_t* cg = malloc((size_t)cap * 2);
    for (uint32_t s = 0; s < cap; ++s) {
        all[s] = base + s;
        fixed_uuid(s, eids + (size_t)s * 16);                   /* EntityID of the entity in slot s */
        fixed_uuid(s | 0x80000000u, cids + (size_t)s * 16);     /* ClientID of its client           */
        on[s] = 1;                                              /* SetClientSyncing(true)           */
        if (gates[s]) { cs[nc] = base + s; cg[nc] = gates[s]; ++nc; }
    }
    check(gw_set_entity_ids(g, all, eids, cap), "gw_set_entity_ids");
    check(gw_set_client_ids(g, all, cids, cap), "gw_set_client_ids");
    check(gw_set_clients(g, cs, cg, nc), "gw_set_clients");
    check(gw_set_client_syncing(g, all, on, cap), "gw_set_client_syncing");
    for (uint32_t i = 0; i < n_init; ++i) slots[i] += base;
    check(gw_space_restore(g, sid, slots, x, y, z, yaw, n_init, GW_SIF_OWN_CLIENT | GW_SIF_NEIGHBOR_CLIENTS),
          "gw_space_restore");

    uint32_t applied_total = 0;
    for (uint32_t t = 0; t < n_ticks; ++t) {
        uint32_t n;
        rd(&n, 4, in);
        gw_op* ops = malloc((size_t)(n ? n : 1) * sizeof(gw_op));
        rd(ops, (size_t)n * sizeof(gw_op), in);
        uint8_t* pkt = malloc((size_t)(n ? n : 1) * 32);
        for (uint32_t i = 0; i < n;) {                          /* runs of one kind, in call order */
            uint32_t j = i;
            if (is_client_move(&ops[i])) {
                while (j < n && is_client_move(&ops[j])) {
                    uint8_t* r = pkt + (size_t)(j - i) * 32;
                    memcpy(r, eids + (size_t)(ops[j].slot) * 16, 16);
                    memcpy(r + 16, &ops[j].x, 4); memcpy(r + 20, &ops[j].y, 4);
                    memcpy(r + 24, &ops[j].z, 4); memcpy(r + 28, &ops[j].yaw, 4);
                    ++j;
                }
                uint32_t applied = 0, to_caller = 0;
                check(gw_submit_client_sync(g, pkt, j - i, &applied, &to_caller), "gw_submit_client_sync");
                if (to_caller) {
                    fprintf(stderr, "c_harness: %u client records left to the caller\n", to_caller);
                    return 2;
                }
                applied_total += applied;
            } else {
                while (j < n && !is_client_move(&ops[j])) ++j;
                for (uint32_t k = i; k < j; ++k) ops[k].slot += base;
                check(gw_submit(g, ops + i, j - i), "gw_submit");
            }
            i = j;
        }
        gw_tick_out to;
        check(gw_tick(g, GW_TICK_COPY_TO_HOST, &to), "gw_tick");
        fwrite(&to.n_enter, 8, 1, out);
        if (to.n_enter) fwrite(to.enter, sizeof(gw_event), to.n_enter, out);
        fwrite(&to.n_leave, 8, 1, out);
        if (to.n_leave) fwrite(to.leave, sizeof(gw_event), to.n_leave, out);
        gw_sync_out so;
        check(gw_sync_collect(g, 0, &so), "gw_sync_collect");
        gw_wire_out wo;
        check(gw_sync_encode_wire(g, GW_WIRE_COPY_TO_HOST, &wo), "gw_sync_encode_wire");
        fwrite(&wo.n_bytes, 8, 1, out);
        if (wo.n_bytes) fwrite(wo.bytes, 1, wo.n_bytes, out);
        fwrite(&wo.n_packets, 4, 1, out);                       /* one packet per gate with records */
        for (uint32_t k = 0; k < wo.n_packets; ++k) {
            const uint32_t gate = wo.gate[k];
            fwrite(&gate, 4, 1, out);
            fwrite(&wo.off[k], 8, 1, out);
        }
        free(ops);
        free(pkt);
    }
    fwrite(&applied_total, 4, 1, out);
    fclose(out);
    fclose(in);
    gw_shutdown(g);
    return 0;
}
