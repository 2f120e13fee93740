// wire.cpp — the host boundary rows of the path:
// entity / client ids of slots, the decode of client position records into
// Moved ops, and the game->gate sync packet encode (on the device).
//
//   a13  GameService.HandleSyncPositionYawFromClient (GameService.go:395-407)
//        -> entity.OnSyncPositionYawFromClient (EntityManager.go:450-459)
//        -> Entity.syncPositionYawFromClient (Entity.go:430-435)
//        -> setPositionYaw(pos, yaw, fromClient=true) (Entity.go:1189-1205)
//   a14  CollectEntitySyncInfos' per-gate packets (Entity.go:1210-1266):
//        Packet.AppendUint16 / AppendClientID / AppendEntityID / AppendFloat32
//        (netutil/Packet.go:66-91,143-162), little-endian (netutil.go:15)
//
// The decode is host work like the reference's (one map lookup per record,
// here an unordered_map of 16-byte ids); its ops join the tick through the
// same validated path as gw_submit, so a record sees the entity's presence as
// of the calls before it.  The encode writes ~48 B per record (hundreds of MB
// at the 1M config): HBM-bound byte work on the device, one thread per output
// dword.
#include <cmath>
#include <cstring>

#include "ctx.hpp"

using namespace gw;
using namespace gw::host;

extern "C" {

int gw_set_entity_ids(gw_ctx* c, const uint32_t* slots, const void* ids, uint32_t n) {
    if (!c || (n && (!slots || !ids))) return GW_EINVAL;
    if (!n) return 0;
    for (uint32_t i = 0; i < n; ++i)
        if (slots[i] >= c->total_slots) return set_err(c, GW_ERANGE, "slot %u out of range", slots[i]);
    if (int rs = settle(c)) return rs;
    (void)hipSetDevice(c->dev);
    const uint8_t* b = (const uint8_t*)ids;
    // a batch names each slot and each (non-zero) id at most once
    std::unordered_map<uint32_t, uint32_t> slot_at;
    std::unordered_map<Id16, uint32_t, Id16Hash> id_at;
    for (uint32_t i = 0; i < n; ++i) {
        if (!slot_at.emplace(slots[i], i).second)
            return set_err(c, GW_EINVAL, "slot %u named twice in one batch", slots[i]);
        const Id16 k = id16(b + (size_t)i * GW_ID_BYTES);
        if ((k.a | k.b) && !id_at.emplace(k, i).second)
            return set_err(c, GW_EINVAL, "entity id of record %u repeated in one batch", i);
    }
    // an id that moves to a new slot is cleared at its old slot (on the device
    // too: the wire encode must never emit one id for two entities)
    std::vector<uint32_t> moved_from;
    for (uint32_t i = 0; i < n; ++i) {
        const Id16 k = id16(b + (size_t)i * GW_ID_BYTES);
        if (!(k.a | k.b)) continue;
        auto it = c->id_slot.find(k);
        if (it != c->id_slot.end() && it->second != slots[i] && !slot_at.count(it->second))
            moved_from.push_back(it->second);
    }
    // device first: a failure leaves host and device as they were
    const uint32_t nt = n + (uint32_t)moved_from.size();
    int rc;
    const size_t off = ((size_t)nt * 4 + 15) & ~(size_t)15;
    if ((rc = ensure(c, c->id_up, off + (size_t)nt * 16))) return rc;
    std::vector<uint32_t> all_slots(slots, slots + n);
    all_slots.insert(all_slots.end(), moved_from.begin(), moved_from.end());
    std::vector<uint8_t> all_ids((size_t)nt * 16, 0);
    memcpy(all_ids.data(), ids, (size_t)n * 16);
    HIPCHK(hipMemcpyAsync(c->id_up.p, all_slots.data(), (size_t)nt * 4, hipMemcpyHostToDevice, c->st));
    HIPCHK(hipMemcpyAsync(P<uint8_t>(c->id_up) + off, all_ids.data(), (size_t)nt * 16, hipMemcpyHostToDevice, c->st));
    launch_put16(c->eid_dev, P<uint32_t>(c->id_up), (const uint4*)(P<uint8_t>(c->id_up) + off), nt, c->st);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(c->st));            // the host arrays are the caller's
    for (uint32_t s : moved_from) c->eid_h[s] = Id16{0, 0};
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t s = slots[i];
        const Id16 old = c->eid_h[s];
        if (old.a | old.b) {
            auto it = c->id_slot.find(old);
            if (it != c->id_slot.end() && it->second == s) c->id_slot.erase(it);
        }
    }
    for (uint32_t i = 0; i < n; ++i) {
        const Id16 k = id16(b + (size_t)i * GW_ID_BYTES);
        c->eid_h[slots[i]] = k;
        if (k.a | k.b) c->id_slot[k] = slots[i];
    }
    return 0;
}

int gw_clear_entity_ids(gw_ctx* c, const uint32_t* slots, uint32_t n) {
    if (!c || (n && !slots)) return GW_EINVAL;
    if (!n) return 0;
    std::vector<uint8_t> zero((size_t)n * 16, 0);
    for (uint32_t i = 0; i < n; ++i) {
        if (slots[i] >= c->total_slots) return set_err(c, GW_ERANGE, "slot %u out of range", slots[i]);
        const Id16 old = c->eid_h[slots[i]];
        auto it = c->id_slot.find(old);
        if ((old.a | old.b) && it != c->id_slot.end() && it->second == slots[i]) c->id_slot.erase(it);
    }
    if (int rc = gw_set_entity_ids(c, slots, zero.data(), n)) return rc;
    c->id_slot.erase(Id16{0, 0});                      // the zero id never maps
    for (uint32_t i = 0; i < n; ++i) c->eid_h[slots[i]] = Id16{0, 0};
    return 0;
}

int gw_set_client_ids(gw_ctx* c, const uint32_t* slots, const void* ids, uint32_t n) {
    if (!c || (n && (!slots || !ids))) return GW_EINVAL;
    if (!n) return 0;
    for (uint32_t i = 0; i < n; ++i)
        if (slots[i] >= c->total_slots) return set_err(c, GW_ERANGE, "slot %u out of range", slots[i]);
    if (int rs = settle(c)) return rs;
    (void)hipSetDevice(c->dev);
    int rc;
    const size_t off = ((size_t)n * 4 + 15) & ~(size_t)15;
    if ((rc = ensure(c, c->id_up, off + (size_t)n * 16))) return rc;
    HIPCHK(hipMemcpyAsync(c->id_up.p, slots, (size_t)n * 4, hipMemcpyHostToDevice, c->st));
    HIPCHK(hipMemcpyAsync(P<uint8_t>(c->id_up) + off, ids, (size_t)n * 16, hipMemcpyHostToDevice, c->st));
    launch_put16(c->cid_dev, P<uint32_t>(c->id_up), (const uint4*)(P<uint8_t>(c->id_up) + off), n, c->st);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(c->st));
    return 0;
}

int gw_set_client_syncing(gw_ctx* c, const uint32_t* slots, const uint8_t* on, uint32_t n) {
    if (!c || (n && (!slots || !on))) return GW_EINVAL;
    for (uint32_t i = 0; i < n; ++i) {
        if (slots[i] >= c->total_slots) return set_err(c, GW_ERANGE, "slot %u out of range", slots[i]);
        c->syncing_h[slots[i]] = on[i] ? 1 : 0;
    }
    return 0;
}

int gw_submit_client_sync(gw_ctx* c, const void* payload, uint32_t n, uint32_t* applied, uint32_t* to_caller) {
    if (!c || (n && !payload)) return GW_EINVAL;
    if (applied) *applied = 0;
    if (to_caller) *to_caller = 0;
    if (!n) return 0;
    if (!c->validate)
        return set_err(c, GW_ESTATE, "client-sync decode needs the host-validated op path (no device-submitted "
                                     "ops on this context)");
    const uint8_t* p = (const uint8_t*)payload;
    std::vector<gw_op> ops;
    ops.reserve(n);
    uint32_t tc = 0;
    for (uint32_t i = 0; i < n; ++i, p += 32) {
        auto it = c->id_slot.find(id16(p));
        if (it == c->id_slot.end()) continue;          // entity not found, may be destroyed (EntityManager.go:451-455)
        const uint32_t s = it->second;
        if (!c->syncing_h[s]) continue;                // !e.syncingFromClient: ignored (Entity.go:432)
        if (!c->present_h[s]) {                        // not in an AOI space here: the caller's reference path
            ++tc;
            continue;
        }
        gw_op o{};
        o.kind = GW_OP_MOVED;
        o.sync_flags = GW_SIF_NEIGHBOR_CLIENTS;        // fromClient: neighbours only (Entity.go:1199-1204)
        o.slot = s;
        float f[4];
        memcpy(f, p + 16, 16);                         // x y z yaw, little-endian (netutil.go:15)
        o.x = f[0]; o.y = f[1]; o.z = f[2]; o.yaw = f[3];
        ops.push_back(o);
    }
    if (to_caller) *to_caller = tc;
    if (ops.empty()) return 0;
    if (int rc = gw_submit(c, ops.data(), (uint32_t)ops.size())) return rc;
    if (applied) *applied = (uint32_t)ops.size();
    return 0;
}

int gw_sync_encode_wire(gw_ctx* c, uint32_t flags, gw_wire_out* out) {
    if (!c || !out) return GW_EINVAL;
    memset(out, 0, sizeof *out);
    if (int rs = settle(c)) return rs;
    (void)hipSetDevice(c->dev);
    const uint64_t R = c->last_rec ? c->last_R : 0;
    const uint32_t G = (uint32_t)c->gate_off.size() ? (uint32_t)c->gate_off.size() - 1 : 0;
    std::vector<WirePacket> pk;
    c->wire_gate.clear();
    c->wire_off.clear();
    uint64_t bytes = 0;
    for (uint32_t g = 0; g < G && R; ++g) {
        const uint64_t n = c->gate_off[g + 1] - c->gate_off[g];
        if (!n) continue;                              // a packet only for a gate with records (Entity.go:1210-1219)
        WirePacket w{};
        w.rec0 = c->gate_off[g];
        w.nrec = n;
        w.byte_off = bytes;
        w.gate = g;
        pk.push_back(w);
        c->wire_gate.push_back((uint16_t)g);
        c->wire_off.push_back(bytes);
        bytes += 4 + 48 * n;
    }
    c->wire_off.push_back(bytes);
    int rc;
    HIPCHK(hipEventRecord(c->ev_t0, c->st));
    if (!pk.empty()) {
        if ((rc = ensure(c, c->wire_d, bytes)) || (rc = ensure(c, c->wire_tab, pk.size() * sizeof(WirePacket))))
            return rc;
        HIPCHK(hipMemcpyAsync(c->wire_tab.p, pk.data(), pk.size() * sizeof(WirePacket), hipMemcpyHostToDevice, c->st));
        launch_wire_encode(c->last_rec, R, P<WirePacket>(c->wire_tab), (uint32_t)pk.size(), c->eid_dev, c->cid_dev,
                           P<uint32_t>(c->wire_d), c->st);
        HIPCHK(hipGetLastError());
    }
    HIPCHK(hipEventRecord(c->ev_t1, c->st));
    out->bytes_dev = P<uint8_t>(c->wire_d);
    out->n_bytes = bytes;
    out->n_packets = (uint32_t)pk.size();
    out->gate = c->wire_gate.data();
    out->off = c->wire_off.data();
    if ((flags & GW_WIRE_COPY_TO_HOST) && bytes) {
        if ((rc = ensure_host(c, c->wire_h, bytes))) return rc;
        HIPCHK(hipMemcpyAsync(c->wire_h.p, c->wire_d.p, bytes, hipMemcpyDeviceToHost, c->st));
        out->bytes = P<uint8_t>(c->wire_h);
    }
    HIPCHK(hipStreamSynchronize(c->st));
    float ms = 0;
    (void)hipEventElapsedTime(&ms, c->ev_t0, c->ev_t1);
    out->device_us = ms * 1000.0;
    return 0;
}

}  // extern "C"
