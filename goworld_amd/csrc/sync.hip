// sync.hip — gfx950 kernels of CollectEntitySyncInfos (Entity.go:1221-1267),
// neighbour queries (InterestedIn / InterestedBy), client updates and the
// primitive instantiations used by the host code.
//
// A flagged entity e's records are: its own client's (syncInfoFlag bit0 and e
// has a client; also after e left the space with the bit kept), then one per
// neighbour w with a client (bit1, e present), neighbours in the order the
// window walk visits them: grid order ((cell of w, w): deterministic).  The neighbours are evaluated from
// the current grid with the stamp-resolved relation (dev_common.hpp), so no
// list is kept.  Count pass, scan, write pass; records land at their final
// offsets, grouped by gate afterwards with a stable radix sort.
#include "dev_common.hpp"

namespace gw {

// ---------------------------------------------------------------------------
// neighbours of a present entity e from the current grid: calls
// f(rel, w, client) per lane for every candidate (rel: w != e is related to e;
// client: w's grid-entry bits CLIENT_BIT | gate id < 16, 0 without a client).
// The window's row ranges are walked flattened, NB_U chunks of 64 in flight.
// (wave_neighbors_of: e's state a and its space P already loaded)
template <int NB_U = 4, typename F>
__device__ __forceinline__ void wave_neighbors_of(const World& w, uint32_t e, const AoiEnt& a, const SpaceP& P, F f) {
    const float d = P.d;
    const Win we = win_of(a.x, a.z, d);
    Rects R;
    R.n = 1;
    R.r[0] = search_rect(P, a.x, a.z);
    Flat fl = flat_build<1>(P, R, w.gn_start, nullptr);
    unsigned long long se = 0;
    bool have_se = false;
    for (uint32_t base = 0; base < fl.total; base += 64u * NB_U) {
        uint32_t idx[NB_U], kd[NB_U];
        flat_map_walk<NB_U, 1>(fl, base, idx, kd);
        GEnt gg[NB_U];
#pragma unroll
        for (int u = 0; u < NB_U; ++u) {
            gg[u].slot = e;
            if (idx[u] != ~0u) gg[u] = w.gn[idx[u]];
        }
#pragma unroll
        for (int u = 0; u < NB_U; ++u) {
            if (base + 64u * u >= fl.total) break;            // wave-uniform
            bool rel = false;
            const GEnt g = gg[u];
            if (g.slot != e) {
                bool ia, near;
                we.test(g.x, g.z, ia, near);              // B's test of A only in the rounding band
                rel = ia;
                if (near) {
                    const bool ib = in_win(g.x, g.z, d, a.x, a.z);
                    if (ia != ib) {
                        if (!have_se) { se = w.rec[e].stamp; have_se = true; }
                        rel = resolve(ia, ib, se, w.rec[g.slot].stamp);
                    }
                }
            }
            f(rel, g.slot, g.meta & (CLIENT_BIT | GATE_MASK));
        }
    }
}
template <int NB_U = 4, typename F>
__device__ __forceinline__ void wave_neighbors(const World& w, uint32_t e, F f) {
    const AoiEnt a = w.rec[e].a;
    if (!(a.meta & PRESENT_BIT)) return;
    wave_neighbors_of<NB_U>(w, e, a, w.sp[a.meta & SPACE_MASK], f);
}

// ---------------------------------------------------------------------------
// flagged entities in slot order, by a one-launch stream compaction (decoupled
// look-back, prim.hpp) of the packed flag words (16 slots each): flagged[k] =
// slot, fbits[k] = its syncInfoFlag.  The flags are cleared here, so the write
// pass reads fbits and can be rerun after the record buffer overflowed.
template <int IPT>
__global__ void __launch_bounds__(NT) k_flag_compact1(uint32_t* __restrict__ flags, uint32_t nwords,
                                                      uint32_t* __restrict__ flagged, uint32_t* __restrict__ fbits,
                                                      unsigned long long* __restrict__ status,
                                                      unsigned long long* __restrict__ ticket,
                                                      unsigned long long tbase, uint32_t tag,
                                                      unsigned long long* total, unsigned long long* ovf,
                                                      uint32_t* __restrict__ zero, uint32_t nzero) {
    __shared__ uint32_t lds[IPT * NWAVE];
    __shared__ uint32_t s_tile, s_prefix;
    if (blockIdx.x == 0 && threadIdx.x == 0) *ovf = 0;
    if (threadIdx.x == 0) s_tile = (uint32_t)(atomicAdd(ticket, 1ull) - tbase);
    __syncthreads();
    const uint32_t tile = s_tile;
    const uint64_t t0 = (uint64_t)tile * (IPT * NT);
    uint32_t f[IPT], c[IPT];
#pragma unroll
    for (int j = 0; j < IPT; ++j) {       // striped: coalesced loads
        const uint64_t i = t0 + (uint64_t)j * NT + threadIdx.x;
        f[j] = i < nwords ? flags[i] : 0u;
        c[j] = (uint32_t)__popc((f[j] | (f[j] >> 1)) & 0x55555555u);   // slots with a bit set
    }
    uint32_t tot;
    tile_excl_scan_striped<uint32_t, IPT>(c, lds, tot);
    if (threadIdx.x < 64) {
        const uint32_t excl = scan_lookback<uint32_t>(status, tile, tag, tot);
        if (threadIdx.x == 0) s_prefix = excl;
    }
    __syncthreads();
    const uint32_t pre = s_prefix;
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        if (f[j]) {
            const uint64_t i = t0 + (uint64_t)j * NT + threadIdx.x;
            uint32_t m = (f[j] | (f[j] >> 1)) & 0x55555555u, at = pre + c[j];
            while (m) {
                const uint32_t b2 = (uint32_t)__builtin_ctz(m);
                m &= m - 1;
                flagged[at] = (uint32_t)(i * 16 + (b2 >> 1));
                fbits[at] = (f[j] >> b2) & 3u;
                ++at;
            }
            flags[i] = 0;
        }
    }
    if (tile == gridDim.x - 1 && threadIdx.x == 0) *total = pre + tot;   // all 64 bits (no reset copy)
    // the next pass's per-space ranges start empty (no fill launch of their own)
    for (uint32_t i = blockIdx.x * NT + threadIdx.x; i < nzero; i += gridDim.x * NT) zero[i] = 0;
}

void launch_flag_compact(uint32_t* flags, uint32_t cap, uint32_t* flagged, uint32_t* fbits, ScanCtx& sc,
                         unsigned long long* total, unsigned long long* ovf, uint32_t* zero, uint32_t nzero,
                         hipStream_t s) {
    const uint32_t nwords = (cap + 15) / 16;
    const bool big = nwords > SCAN_BIG;
    const uint64_t tile = big ? 2 * SCAN_TILE : SCAN_TILE;
    uint32_t nb = (uint32_t)((nwords + tile - 1) / tile);
    if (nb == 0) nb = 1;
    if (sc.tag >= SCAN_TAG_MAX) {
        (void)hipMemsetAsync(sc.status, 0, sc.max_tiles * SCAN_WORDS * 8, s);
        sc.tag = 0;
    }
    ++sc.tag;
    if (big)
        hipLaunchKernelGGL(k_flag_compact1<2 * SCAN_IPT>, dim3(nb), dim3(NT), 0, s, flags, nwords, flagged, fbits,
                           sc.status, sc.ticket, sc.tbase, sc.tag, total, ovf, zero, nzero);
    else
        hipLaunchKernelGGL(k_flag_compact1<SCAN_IPT>, dim3(nb), dim3(NT), 0, s, flags, nwords, flagged, fbits,
                           sc.status, sc.ticket, sc.tbase, sc.tag, total, ovf, zero, nzero);
    sc.tbase += nb;
}

// Flagged entities are walked by a capped grid of waves (grid-stride): the
// count lives on the device, so a grid sized for the worst case would
// dispatch mostly empty waves.
constexpr uint32_t SYNC_MAX_BLOCKS = 8192;

// record count per flagged entity: a lane per entity (the diff's cached count
// of neighbours with a client when it is from this epoch); the entities that
// need a window walk are then walked one at a time by the whole wave
// Small-space mode (sfirst non-null): each space's run [sfirst, slast) of the
// flagged list (slot order) for the write pass, from the spaces this pass
// reads anyway; the neighbours' spaces come from the adjacent lanes, only a
// wave's edge lanes gather one more.
template <int U>
__global__ void __launch_bounds__(NT) k_sync_count(World w, const uint32_t* __restrict__ flagged,
                                                   const uint32_t* __restrict__ fbits, const uint64_t* nf_dev,
                                                   uint32_t nf_max, uint32_t* cnt, uint32_t* __restrict__ sfirst,
                                                   uint32_t* __restrict__ slast) {
    const uint64_t nf = load_n(nf_max, nf_dev);
    const int ln = lane_id();
    const uint64_t stride = (uint64_t)gridDim.x * NT;
    for (uint64_t base = (uint64_t)blockIdx.x * NT + (threadIdx.x & ~63u); base < nf; base += stride) {
        const uint64_t k = base + ln;
        const bool valid = k < nf;
        uint32_t e = 0, f = 0, r = 0, gt = 0;
        AoiEnt a{};
        unsigned long long c = 0;
        uint32_t eo = 0xffffffffu;                          // small-space mode: an edge lane's outer neighbour
        if (valid) {
            e = flagged[k];
            f = fbits[k];
        }
        if (sfirst) {                                       // kernel-uniform
            if (ln == 0 && valid && k) eo = flagged[k - 1];
            if (ln == 63 && k + 1 < nf) eo = flagged[k + 1];
        }
        if (valid) {
            a = w.rec[e].a;
            gt = w.rec[e].gate;                             // loaded with the state, not behind the test
            c = w.nbc[e];
        }
        if (sfirst) {
            const uint32_t so = eo != 0xffffffffu ? (w.rec[eo].a.meta & SPACE_MASK) : 0xffffffffu;
            const uint32_t sq = valid ? (a.meta & SPACE_MASK) : 0xffffffffu;
            uint32_t sp = (uint32_t)__shfl_up((int)sq, 1, 64);
            uint32_t sn = (uint32_t)__shfl_down((int)sq, 1, 64);
            if (ln == 0) sp = so;
            if (ln == 63) sn = so;
            if (valid && sp != sq) sfirst[sq] = (uint32_t)k;
            if (valid && sn != sq) slast[sq] = (uint32_t)(k + 1);
        }
        bool walk = false;
        if (valid) {
            // an entity that left the space (into the nil space, keeping its
            // flag) still syncs its own client (Entity.go:1221-1239); only a
            // present one has neighbours
            if (owned_x(w.sp[a.meta & SPACE_MASK], a.x)) {
                if ((f & GW_SIF_OWN_CLIENT) && gt) r = 1;
                if ((f & GW_SIF_NEIGHBOR_CLIENTS) && (a.meta & PRESENT_BIT)) {
                    if ((uint32_t)(c >> 32) == w.epoch) r += (uint32_t)c & NBC_COUNT;   // counted by this tick's diff
                    else walk = true;
                }
            }
        }
        uint64_t todo = wave_ballot(walk);
        while (todo) {
            const int q = __builtin_ctzll(todo);
            todo &= todo - 1;
            const uint32_t eq = (uint32_t)__builtin_amdgcn_readlane((int)e, q);
            uint32_t n = 0;
            wave_neighbors<U>(w, eq, [&](bool rel, uint32_t, uint32_t g) {
                n += (uint32_t)popc64(wave_ballot(rel && g != 0));
            });
            if (ln == q) r += n;
        }
        if (valid) cnt[k] = r;
    }
}
void launch_sync_count(const World& w, const uint32_t* flagged, const uint32_t* fbits, const uint64_t* nf_dev,
                       uint32_t nf_max, uint32_t* cnt, uint32_t* sfirst, uint32_t* slast, hipStream_t s) {
    if (!nf_max) return;
    const dim3 g(std::min(nblk(nf_max, NT), SYNC_MAX_BLOCKS));
    if (w.nb_u >= 8)
        hipLaunchKernelGGL(k_sync_count<8>, g, dim3(NT), 0, s, w, flagged, fbits, nf_dev, nf_max, cnt, sfirst, slast);
    else if (w.nb_u <= 2)
        hipLaunchKernelGGL(k_sync_count<2>, g, dim3(NT), 0, s, w, flagged, fbits, nf_dev, nf_max, cnt, sfirst, slast);
    else
        hipLaunchKernelGGL(k_sync_count<4>, g, dim3(NT), 0, s, w, flagged, fbits, nf_dev, nf_max, cnt, sfirst, slast);
}

// A record as three 8-B non-temporal stores: the collect never reads its
// records back, and streaming them past the caches keeps the grid and state
// the next tick reads resident in L2 (sync_write 148 -> 131 us at config #3,
// grid and diff a few us faster too; the same for the tick's event arrays,
// which the segment fix-up re-reads, was 12 us slower)
__device__ __forceinline__ void st_record_nt(gw_sync_record* r, uint32_t watcher, uint32_t entity, float4 p) {
    unsigned long long* q = (unsigned long long*)r;
    __builtin_nontemporal_store(((unsigned long long)entity << 32) | watcher, q);
    __builtin_nontemporal_store(((unsigned long long)__float_as_uint(p.y) << 32) | __float_as_uint(p.x), q + 1);
    __builtin_nontemporal_store(((unsigned long long)__float_as_uint(p.w) << 32) | __float_as_uint(p.z), q + 2);
}

// The neighbour records of one entity leave through a per-wave LDS buffer
// (SW_BUF records): once 64 are staged they are written as 3 x 64 contiguous
// 8-B non-temporal stores (512 B per instruction) instead of one strided
// 8-B store per record field.
constexpr int SW_BUF = 128;
__device__ __forceinline__ void sw_flush64(unsigned long long* buf, unsigned long long* dst, uint32_t n_rec) {
    const int ln = lane_id();
    const uint32_t words = 3 * n_rec;
#pragma unroll
    for (uint32_t j = 0; j < 3; ++j) {
        const uint32_t i = j * 64 + (uint32_t)ln;
        if (i < words) __builtin_nontemporal_store(buf[i], dst + i);
    }
}

// writes e's records at rec_off[k] (nothing if the buffer is too small: the
// host grows it and reruns this pass).  PAIRS (the per-client grouping): only
// (watcher, entity) as two u32 arrays, the sort's keys and values (pk, pv),
// whose 24-B records are built once after the sort (k_records_from_pairs)
// (GW_SW_MINB: blocks per CU the register allocation must allow; 8 caps the
// VGPRs at 64, i.e. 8 waves per SIMD instead of 7 at 66)
#ifndef GW_SW_MINB
#define GW_SW_MINB 1
#endif
// An entity's header (its flagged-list entry) and state: a wave walks
// entities k, k + stride, ... and loads the next entity's state and the one
// after's header before it walks the current one, so those two dependent
// loads are in flight during the walk instead of ahead of it.
struct SwHdr {
    uint32_t e, f, cnt;
    uint64_t at;
};
struct SwEnt {
    AoiEnt a;
    uint32_t gt;
};
template <int U, bool PAIRS = false>
__global__ void __launch_bounds__(NT, GW_SW_MINB) k_sync_write(World w, const uint32_t* __restrict__ flagged,
                                                   const uint32_t* __restrict__ fbits, const uint64_t* nf_dev,
                                                   uint32_t nf_max, const uint64_t* __restrict__ rec_off,
                                                   const uint32_t* __restrict__ cnt, gw_sync_record* rec,
                                                   uint64_t rec_cap, DevStats* st, uint64_t* __restrict__ pr,
                                                   float4* __restrict__ pay) {
    __shared__ unsigned long long sbuf[NWAVE][3 * SW_BUF];
    unsigned long long* buf = sbuf[threadIdx.x >> 6];
    const uint64_t nf = load_n(nf_max, nf_dev);
    const int ln = lane_id();
    const uint64_t lt = lanemask_lt();
    const uint64_t stride = (uint64_t)gridDim.x * NWAVE;
    auto hdr = [&](uint64_t q) {
        SwHdr h{};
        if (q < nf) {
            h.e = flagged[q];
            h.f = fbits[q];
            h.at = rec_off[q];
            h.cnt = cnt[q];
        }
        return h;
    };
    auto ent = [&](uint64_t q, const SwHdr& h) {
        SwEnt x{};
        if (q < nf) {
            x.a = w.rec[h.e].a;
            x.gt = w.rec[h.e].gate;
        }
        return x;
    };
    auto one = [&](uint64_t k, const SwHdr& h, const SwEnt& x) {
        const uint32_t e = h.e, f = h.f;
        uint64_t at = h.at;
        if (at + h.cnt > rec_cap) {
            if (ln == 0) atomicOr(&st->overflow, 1ull);
            return;
        }
        const AoiEnt a = x.a;
        const float4 p = w.rec[e].p;                          // used at the first record: in flight with the walk
        const SpaceP P = w.sp[a.meta & SPACE_MASK];
        if (!owned_x(P, a.x)) return;
        // PAIRS: the value is the flagged index k, and the entity's payload goes
        // to pay[k]: the records are built from that compact table (L2-resident)
        // instead of a 64-B slot-state line per record
        if (PAIRS && ln == 0) pay[k] = p;
        if ((f & GW_SIF_OWN_CLIENT) && x.gt) {
            if (ln == 0) {
                if (PAIRS) {
                    pr[at] = (k << 32) | e;
                } else {
                    st_record_nt(rec + at, e, e, p);
                }
            }
            ++at;
        }
        if (!(f & GW_SIF_NEIGHBOR_CLIENTS) || !(a.meta & PRESENT_BIT)) return;
        if (PAIRS) {
            wave_neighbors_of<U>(w, e, a, P, [&](bool rel, uint32_t ws, uint32_t g) {
                const bool take = rel && g != 0;
                const uint64_t bt = wave_ballot(take);
                if (take) pr[at + (uint64_t)popc64(bt & lt)] = (k << 32) | ws;
                at += (uint64_t)popc64(bt);
            });
            return;
        }
        const unsigned long long pxy = ((unsigned long long)__float_as_uint(p.y) << 32) | __float_as_uint(p.x);
        const unsigned long long pzw = ((unsigned long long)__float_as_uint(p.w) << 32) | __float_as_uint(p.z);
        uint32_t nb = 0;                                      // staged records (wave-uniform)
        wave_neighbors_of<U>(w, e, a, P, [&](bool rel, uint32_t ws, uint32_t g) {
            const bool take = rel && g != 0;
            const uint64_t bt = wave_ballot(take);
            if (take) {
                unsigned long long* r = buf + 3 * (nb + (uint32_t)popc64(bt & lt));
                r[0] = ((unsigned long long)e << 32) | ws;
                r[1] = pxy;
                r[2] = pzw;
            }
            nb += (uint32_t)popc64(bt);
            if (nb >= 64) {
                wave_sync();
                sw_flush64(buf, (unsigned long long*)(rec + at), 64);
                at += 64;
                nb -= 64;
                wave_sync();
                for (uint32_t i = (uint32_t)ln; i < 3 * nb; i += 64) buf[i] = buf[192 + i];
                wave_sync();
            }
        });
        if (nb) {
            wave_sync();
            sw_flush64(buf, (unsigned long long*)(rec + at), nb);
            wave_sync();
        }
    };
    // the wave index as a uniform value: the headers and states are scalar
    // loads into SGPRs, not VGPRs that would cost the walk its occupancy
    uint64_t k = (uint64_t)blockIdx.x * NWAVE + (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    SwHdr h0 = hdr(k);
    SwEnt x0 = ent(k, h0);
    SwHdr h1 = hdr(k + stride);
    for (; k < nf; k += stride) {
        const SwEnt x1 = ent(k + stride, h1);
        const SwHdr h2 = hdr(k + 2 * stride);
        one(k, h0, x0);
        h0 = h1;
        x0 = x1;
        h1 = h2;
    }
}
// ---------------------------------------------------------------------------
// Short lists two per wave (GW_SW_HALVES): a wave takes flagged entries k and
// k+1; when both have <= SW_HALF_MAX records each half-wave (32 lanes) walks
// its own entity's window (rows and candidates from HBM, a 5-step search over
// the half's row prefixes per 32 candidates) and stores its records directly;
// otherwise both go through the full-wave walk of k_sync_write one after the
// other.  A uniform world (config #5: ~38 records per entity) spends most of
// a full-wave walk on per-entity setup.
constexpr uint32_t SW_HALF_MAX = 64;

template <int U>
__device__ __forceinline__ void sw_full(const World& w, uint32_t e, uint32_t f, uint64_t at, uint32_t c,
                                        gw_sync_record* rec, uint64_t rec_cap, DevStats* st,
                                        unsigned long long* buf) {
    const int ln = lane_id();
    const uint64_t lt = lanemask_lt();
    if (at + c > rec_cap) {
        if (ln == 0) atomicOr(&st->overflow, 1ull);
        return;
    }
    const AoiEnt a = w.rec[e].a;
    const float4 p = w.rec[e].p;
    const uint32_t gt = w.rec[e].gate;
    const SpaceP P = w.sp[a.meta & SPACE_MASK];
    if (!owned_x(P, a.x)) return;
    if ((f & GW_SIF_OWN_CLIENT) && gt) {
        if (ln == 0) st_record_nt(rec + at, e, e, p);
        ++at;
    }
    if (!(f & GW_SIF_NEIGHBOR_CLIENTS) || !(a.meta & PRESENT_BIT)) return;
    const unsigned long long pxy = ((unsigned long long)__float_as_uint(p.y) << 32) | __float_as_uint(p.x);
    const unsigned long long pzw = ((unsigned long long)__float_as_uint(p.w) << 32) | __float_as_uint(p.z);
    uint32_t nb = 0;
    wave_neighbors_of<U>(w, e, a, P, [&](bool rel, uint32_t ws, uint32_t g) {
        const bool take = rel && g != 0;
        const uint64_t bt = wave_ballot(take);
        if (take) {
            unsigned long long* r = buf + 3 * (nb + (uint32_t)popc64(bt & lt));
            r[0] = ((unsigned long long)e << 32) | ws;
            r[1] = pxy;
            r[2] = pzw;
        }
        nb += (uint32_t)popc64(bt);
        if (nb >= 64) {
            wave_sync();
            sw_flush64(buf, (unsigned long long*)(rec + at), 64);
            at += 64;
            nb -= 64;
            wave_sync();
            for (uint32_t i = (uint32_t)ln; i < 3 * nb; i += 64) buf[i] = buf[192 + i];
            wave_sync();
        }
    });
    if (nb) {
        wave_sync();
        sw_flush64(buf, (unsigned long long*)(rec + at), nb);
        wave_sync();
    }
}

// (GW_SWH_MINB 8 caps it at 64 VGPRs, 8 waves per SIMD instead of 7 at 66,
// but spills 2 VGPRs to scratch: config #5 write 851 -> 907-930 us; uncapped)
#ifndef GW_SWH_MINB
#define GW_SWH_MINB 1
#endif
template <int U>
__global__ void __launch_bounds__(NT, GW_SWH_MINB) k_sync_write_h(World w, const uint32_t* __restrict__ flagged,
                                                     const uint32_t* __restrict__ fbits, const uint64_t* nf_dev,
                                                     uint32_t nf_max, const uint64_t* __restrict__ rec_off,
                                                     const uint32_t* __restrict__ cnt, gw_sync_record* rec,
                                                     uint64_t rec_cap, DevStats* st) {
    __shared__ unsigned long long sbuf[NWAVE][3 * SW_BUF];
    unsigned long long* buf = sbuf[threadIdx.x >> 6];
    const uint64_t nf = load_n(nf_max, nf_dev);
    const int ln = lane_id();
    const uint32_t half = (uint32_t)ln >> 5, hl = (uint32_t)ln & 31u, hb = half << 5;
    const uint64_t hmask = half ? 0xffffffff00000000ull : 0x00000000ffffffffull;
    const uint64_t lt = lanemask_lt();
    const uint64_t stride = (uint64_t)gridDim.x * NWAVE * 2;
    for (uint64_t k0 = ((uint64_t)blockIdx.x * NWAVE + (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6))) * 2;
         k0 < nf; k0 += stride) {
        const bool hasB = k0 + 1 < nf;
        const uint32_t cA = cnt[k0], cB = hasB ? cnt[k0 + 1] : 0u;
        if (max(cA, cB) > SW_HALF_MAX) {                       // wave-uniform: full-wave walks
            sw_full<U>(w, flagged[k0], fbits[k0], rec_off[k0], cA, rec, rec_cap, st, buf);
            if (hasB) {
                wave_sync();
                sw_full<U>(w, flagged[k0 + 1], fbits[k0 + 1], rec_off[k0 + 1], cB, rec, rec_cap, st, buf);
            }
            continue;
        }
        const uint64_t k = k0 + half;
        const bool valid = k < nf;
        uint32_t e = 0, f = 0, c = 0;
        uint64_t at = 0;
        if (valid) {
            e = flagged[k];
            f = fbits[k];
            at = rec_off[k];
            c = half ? cB : cA;
        }
        AoiEnt a;
        a.x = a.z = 0.0f;
        a.meta = 0;
        float4 p = make_float4(0.f, 0.f, 0.f, 0.f);
        uint32_t gt = 0;
        if (valid) {
            a = w.rec[e].a;
            p = w.rec[e].p;
            gt = w.rec[e].gate;
        }
        const SpaceP P = w.sp[a.meta & SPACE_MASK];
        bool walk = false;
        if (valid) {
            if (at + c > rec_cap) {
                if (hl == 0) atomicOr(&st->overflow, 1ull);
            } else if (owned_x(P, a.x)) {
                if ((f & GW_SIF_OWN_CLIENT) && gt) {
                    if (hl == 0) st_record_nt(rec + at, e, e, p);
                    ++at;
                }
                walk = (f & GW_SIF_NEIGHBOR_CLIENTS) && (a.meta & PRESENT_BIT);
            }
        }
        // the half's row ranges (lane hl: row hl of its window), then its scan
        const float d = P.d;
        uint32_t rs = 0, rl = 0;
        const Win we = win_of(a.x, a.z, d);
        if (walk) {
            const Rect r = search_rect(P, a.x, a.z);
            const int nr = r.z1 - r.z0 + 1;
            if ((int)hl < nr) {
                const uint32_t base = P.cell_base + (uint32_t)(r.z0 + (int)hl) * (uint32_t)P.W;
                rs = w.gn_start[base + (uint32_t)r.x0];
                rl = w.gn_start[base + (uint32_t)r.x1 + 1] - rs;
            }
        }
        const uint32_t inc64 = wave_incl_scan<uint32_t>(rl);
        const uint32_t lo31 = (uint32_t)__builtin_amdgcn_readlane((int)inc64, 31);
        const uint32_t inc = half ? inc64 - lo31 : inc64;
        const uint32_t pre = inc - rl;
        const uint32_t tot0 = lo31, tot1 = (uint32_t)__builtin_amdgcn_readlane((int)inc64, 63) - lo31;
        const uint32_t total = half ? tot1 : tot0;
        const uint32_t tmax = max(tot0, tot1);
        const unsigned long long pxy = ((unsigned long long)__float_as_uint(p.y) << 32) | __float_as_uint(p.x);
        const unsigned long long pzw = ((unsigned long long)__float_as_uint(p.w) << 32) | __float_as_uint(p.z);
        unsigned long long se = 0;
        bool have_se = false;
        for (uint32_t B = 0; B < tmax; B += 32) {              // wave-uniform
            const uint32_t kk = B + hl;
            uint32_t l2 = 0;
#pragma unroll
            for (int step = 16; step; step >>= 1) {
                const uint32_t cc = l2 + (uint32_t)step;
                const uint32_t pv = (uint32_t)__shfl((int)pre, (int)(hb + min(cc, 31u)), 64);
                if (cc < 32u && pv <= kk) l2 = cc;
            }
            const uint32_t ss = (uint32_t)__shfl((int)rs, (int)(hb + l2), 64);
            const uint32_t sp = (uint32_t)__shfl((int)pre, (int)(hb + l2), 64);
            bool take = false;
            GEnt g;
            g.slot = e;
            g.meta = 0;
            if (kk < total) g = w.gn[ss + (kk - sp)];
            if (kk < total && g.slot != e && (g.meta & CLIENT_BIT)) {
                bool ia, near;
                we.test(g.x, g.z, ia, near);              // B's test of A only in the rounding band
                bool rel = ia;
                if (near) {
                    const bool ib = in_win(g.x, g.z, d, a.x, a.z);
                    if (ia != ib) {
                        if (!have_se) { se = w.rec[e].stamp; have_se = true; }
                        rel = resolve(ia, ib, se, w.rec[g.slot].stamp);
                    }
                }
                take = rel;
            }
            const uint64_t bt = wave_ballot(take) & hmask;
            if (take) {
                unsigned long long* q = (unsigned long long*)(rec + at + (uint64_t)popc64(bt & lt));
                __builtin_nontemporal_store(((unsigned long long)e << 32) | g.slot, q);
                __builtin_nontemporal_store(pxy, q + 1);
                __builtin_nontemporal_store(pzw, q + 2);
            }
            at += (uint64_t)popc64(bt);
        }
    }
}

// ---------------------------------------------------------------------------
// Small-space mode (every space's grid fits in LDS, e.g. config #4's 10k
// spaces of 1k): one block per space loads the space's grid entries and row
// starts into LDS once, then its waves write the records of the space's
// flagged entities (a contiguous range of the slot-ordered flagged list) with
// every candidate read from LDS: the per-entity chain of dependent global
// loads shrinks to the entity's own state.
template <int NB_U, typename F>
__device__ __forceinline__ void wave_neighbors_lds(const World& w, uint32_t e, const AoiEnt& a, const SpaceP& P,
                                                   const GEnt* G, uint32_t g0, const uint32_t* S, F f) {
    const float d = P.d;
    const Win we = win_of(a.x, a.z, d);
    Rects R;
    R.n = 1;
    R.r[0] = search_rect(P, a.x, a.z);
    Flat fl = flat_build<1>(P, R, S - P.cell_base, nullptr);   // S[c - cell_base] = gn_start[c]
    unsigned long long se = 0;
    bool have_se = false;
    for (uint32_t base = 0; base < fl.total; base += 64u * NB_U) {
        uint32_t idx[NB_U], kd[NB_U];
        flat_map<NB_U, 1>(fl, base, idx, kd);
#pragma unroll
        for (int u = 0; u < NB_U; ++u) {
            if (base + 64u * u >= fl.total) break;            // wave-uniform
            bool rel = false;
            GEnt g;
            g.slot = e;
            g.meta = 0;
            if (idx[u] != ~0u) g = G[idx[u] - g0];
            if (g.slot != e) {
                bool ia, near;
                we.test(g.x, g.z, ia, near);              // B's test of A only in the rounding band
                rel = ia;
                if (near) {
                    const bool ib = in_win(g.x, g.z, d, a.x, a.z);
                    if (ia != ib) {
                        if (!have_se) { se = w.rec[e].stamp; have_se = true; }
                        rel = resolve(ia, ib, se, w.rec[g.slot].stamp);
                    }
                }
            }
            f(rel, g.slot, g.meta & (CLIENT_BIT | GATE_MASK));
        }
    }
}

template <int U>
__global__ void __launch_bounds__(NT) k_sync_write_small(World w, const uint32_t* __restrict__ flagged,
                                                         const uint32_t* __restrict__ fbits,
                                                         const uint64_t* __restrict__ rec_off,
                                                         const uint32_t* __restrict__ cnt, gw_sync_record* rec,
                                                         uint64_t rec_cap, DevStats* st,
                                                         const uint32_t* __restrict__ sfirst,
                                                         const uint32_t* __restrict__ slast, uint32_t max_ents) {
    extern __shared__ uint4 dyn_lds[];
    const uint32_t s = blockIdx.x;
    const uint32_t lo = sfirst[s], hi = slast[s];
    if (lo >= hi) return;                                   // block-uniform
    const SpaceP P = w.sp[s];
    const uint32_t cb = P.cell_base, nc = (uint32_t)(P.W * P.H);
    const uint32_t g0 = w.gn_start[cb], g1 = w.gn_start[cb + nc];
    GEnt* G = (GEnt*)dyn_lds;
    uint32_t* S = (uint32_t*)(G + max_ents);
    const uint32_t ng = min(g1 - g0, max_ents);             // (host guarantee: g1 - g0 <= max_ents)
    lds_fill16<NT>((uint4*)G, (const uint4*)(w.gn + g0), ng);
    for (uint32_t i = threadIdx.x; i <= nc; i += NT) S[i] = w.gn_start[cb + i];
    __syncthreads();
    const int ln = lane_id();
    const uint64_t lt = lanemask_lt();
    for (uint32_t k = lo + (threadIdx.x >> 6); k < hi; k += NWAVE) {
        const uint32_t e = flagged[k];
        const uint32_t f = fbits[k];
        uint64_t at = rec_off[k];
        if (at + cnt[k] > rec_cap) {
            if (ln == 0) atomicOr(&st->overflow, 1ull);
            continue;
        }
        const AoiEnt a = w.rec[e].a;
        if (!owned_x(P, a.x)) continue;
        const float4 p = w.rec[e].p;
        if ((f & GW_SIF_OWN_CLIENT) && w.rec[e].gate) {
            if (ln == 0) st_record_nt(rec + at, e, e, p);
            ++at;
        }
        if ((f & GW_SIF_NEIGHBOR_CLIENTS) && (a.meta & PRESENT_BIT)) {
            wave_neighbors_lds<U>(w, e, a, P, G, g0, S, [&](bool rel, uint32_t ws, uint32_t g) {
                const bool take = rel && g != 0;
                const uint64_t bt = wave_ballot(take);
                if (take) st_record_nt(rec + at + (uint64_t)popc64(bt & lt), ws, e, p);
                at += (uint64_t)popc64(bt);
            });
        }
    }
}

// The same with two entities per wave (a half-wave each): with short
// candidate lists (config #4: ~80) the per-entity setup dominates a wave's
// VALU, and a half-wave still covers a list in 2-3 chunks of 32.  Rows of a
// window (<= 11) fit a half-wave; the row scan is the wave scan minus lane
// 31's prefix for the upper half; a lane finds its range by a 5-step search
// over its half's prefixes; record slots come from the half's ballot bits.
__global__ void __launch_bounds__(NT) k_sync_write_small2(World w, const uint32_t* __restrict__ flagged,
                                                          const uint32_t* __restrict__ fbits,
                                                          const uint64_t* __restrict__ rec_off,
                                                          const uint32_t* __restrict__ cnt, gw_sync_record* rec,
                                                          uint64_t rec_cap, DevStats* st,
                                                          const uint32_t* __restrict__ sfirst,
                                                          const uint32_t* __restrict__ slast, uint32_t max_ents) {
    extern __shared__ uint4 dyn_lds[];
    const uint32_t s = blockIdx.x;
    const uint32_t lo = sfirst[s], hi = slast[s];
    if (lo >= hi) return;                                   // block-uniform
    const SpaceP P = w.sp[s];
    const uint32_t cb = P.cell_base, nc = (uint32_t)(P.W * P.H);
    const uint32_t g0 = w.gn_start[cb], g1 = w.gn_start[cb + nc];
    GEnt* G = (GEnt*)dyn_lds;
    uint32_t* S = (uint32_t*)(G + max_ents);
    const uint32_t ng = min(g1 - g0, max_ents);
    lds_fill16<NT>((uint4*)G, (const uint4*)(w.gn + g0), ng);
    for (uint32_t i = threadIdx.x; i <= nc; i += NT) S[i] = w.gn_start[cb + i];
    __syncthreads();
    const int ln = lane_id();
    const uint32_t half = (uint32_t)ln >> 5, hl = (uint32_t)ln & 31u, hb = half << 5;
    const uint64_t hmask = half ? 0xffffffff00000000ull : 0x00000000ffffffffull;
    const uint64_t lt = lanemask_lt();
    const float d = P.d;
    // the entity's list entry, then its state: position and gate are loaded
    // with the AOI state (not behind the ownership test)
    const auto entry = [&](uint32_t k, uint32_t& e, uint32_t& f, uint64_t& at, uint32_t& c) {
        e = f = c = 0;
        at = 0;
        if (k < hi) { e = flagged[k]; f = fbits[k]; at = rec_off[k]; c = cnt[k]; }
    };
    // the next pair's states are loaded during this pair's walks and its list
    // entries two pairs ahead (config #4 write 430 -> 422 us; the same in
    // k_sync_write_h took it from 66 to 92 VGPRs and the 16M world's write
    // from 852 to 976 us)
    struct SwSt {
        AoiEnt a;
        float4 p;
        uint32_t gt;
    };
    const auto state = [&](uint32_t k, uint32_t e, SwSt& x) {
        x.a.x = x.a.z = 0.0f;
        x.a.meta = 0;
        x.p = make_float4(0, 0, 0, 0);
        x.gt = 0;
        if (k < hi) {
            x.a = w.rec[e].a;
            x.p = w.rec[e].p;
            x.gt = w.rec[e].gate;
        }
    };
    constexpr uint32_t STEP = NWAVE * 2;
    const uint32_t kfirst = lo + (threadIdx.x >> 6) * 2;
    uint32_t ne, nf, nc_, ne2, nf2, nc2;
    uint64_t nat, nat2;
    entry(kfirst + half, ne, nf, nat, nc_);
    entry(kfirst + STEP + half, ne2, nf2, nat2, nc2);
    SwSt nst;
    state(kfirst + half, ne, nst);
    for (uint32_t k0 = kfirst; k0 < hi; k0 += STEP) {
        const uint32_t k = k0 + half;
        const bool valid = k < hi;
        const uint32_t e = ne, f = nf, c = nc_;
        uint64_t at = nat;
        const SwSt cs = nst;
        ne = ne2; nf = nf2; nat = nat2; nc_ = nc2;
        entry(k0 + 2 * STEP + half, ne2, nf2, nat2, nc2);
        state(k0 + STEP + half, ne, nst);
        bool walk = false;
        const AoiEnt a = cs.a;
        const float4 p = cs.p;
        const uint32_t gt = cs.gt;
        if (valid) {
            if (at + c > rec_cap) {
                if (hl == 0) atomicOr(&st->overflow, 1ull);
            } else {
                if (owned_x(P, a.x)) {
                    if ((f & GW_SIF_OWN_CLIENT) && gt) {
                        if (hl == 0) st_record_nt(rec + at, e, e, p);
                        ++at;
                    }
                    walk = (f & GW_SIF_NEIGHBOR_CLIENTS) && (a.meta & PRESENT_BIT);
                }
            }
        }
        // the half's row ranges (lane hl: row hl of its window), then its scan
        uint32_t rs = 0, rl = 0;
        const Win we = win_of(a.x, a.z, d);
        if (walk) {
            const Rect r = search_rect(P, a.x, a.z);
            const int nr = r.z1 - r.z0 + 1;
            if ((int)hl < nr) {
                const uint32_t base = (uint32_t)(r.z0 + (int)hl) * (uint32_t)P.W;   // local cell index
                rs = S[base + (uint32_t)r.x0];
                rl = S[base + (uint32_t)r.x1 + 1] - rs;
            }
        }
        const uint32_t inc64 = wave_incl_scan<uint32_t>(rl);
        const uint32_t lo31 = (uint32_t)__builtin_amdgcn_readlane((int)inc64, 31);
        const uint32_t inc = half ? inc64 - lo31 : inc64;
        const uint32_t pre = inc - rl;
        const uint32_t tot0 = lo31, tot1 = (uint32_t)__builtin_amdgcn_readlane((int)inc64, 63) - lo31;
        const uint32_t total = half ? tot1 : tot0;
        const uint32_t tmax = max(tot0, tot1);
        const unsigned long long pxy = ((unsigned long long)__float_as_uint(p.y) << 32) | __float_as_uint(p.x);
        const unsigned long long pzw = ((unsigned long long)__float_as_uint(p.w) << 32) | __float_as_uint(p.z);
        unsigned long long se = 0;
        bool have_se = false;
        for (uint32_t B = 0; B < tmax; B += 32) {             // wave-uniform
            const uint32_t kk = B + hl;
            uint32_t l2 = 0;
#pragma unroll
            for (int step = 16; step; step >>= 1) {
                const uint32_t cc = l2 + (uint32_t)step;
                const uint32_t pv = (uint32_t)__shfl((int)pre, (int)(hb + min(cc, 31u)), 64);
                if (cc < 32u && pv <= kk) l2 = cc;
            }
            const uint32_t ss = (uint32_t)__shfl((int)rs, (int)(hb + l2), 64);
            const uint32_t sp = (uint32_t)__shfl((int)pre, (int)(hb + l2), 64);
            bool take = false;
            GEnt g;
            g.slot = e;
            g.meta = 0;
            if (kk < total) g = G[ss + (kk - sp) - g0];
            if (kk < total && g.slot != e && (g.meta & CLIENT_BIT)) {
                bool ia, near;
                we.test(g.x, g.z, ia, near);              // B's test of A only in the rounding band
                bool rel = ia;
                if (near) {
                    const bool ib = in_win(g.x, g.z, d, a.x, a.z);
                    if (ia != ib) {
                        if (!have_se) { se = w.rec[e].stamp; have_se = true; }
                        rel = resolve(ia, ib, se, w.rec[g.slot].stamp);
                    }
                }
                take = rel;
            }
            const uint64_t bt = wave_ballot(take) & hmask;
            if (take) {
                unsigned long long* q = (unsigned long long*)(rec + at + (uint64_t)popc64(bt & lt));
                __builtin_nontemporal_store(((unsigned long long)e << 32) | g.slot, q);
                __builtin_nontemporal_store(pxy, q + 1);
                __builtin_nontemporal_store(pzw, q + 2);
            }
            at += (uint64_t)popc64(bt);
        }
    }
}

void launch_sync_write_small(const World& w, uint32_t n_spaces, const uint32_t* flagged, const uint32_t* fbits,
                             const uint64_t* rec_off, const uint32_t* cnt, gw_sync_record* rec, uint64_t rec_cap,
                             DevStats* st, const uint32_t* sfirst, const uint32_t* slast, uint32_t max_ents,
                             uint32_t max_cells, hipStream_t s) {
    if (!n_spaces) return;
    const size_t lds = (size_t)max_ents * sizeof(GEnt) + ((size_t)max_cells + 1) * 4;
    static const bool halves = !getenv("GW_SYNC_HALVES") || atoi(getenv("GW_SYNC_HALVES")) != 0;
    if (halves) {
        hipLaunchKernelGGL(k_sync_write_small2, dim3(n_spaces), dim3(NT), lds, s, w, flagged, fbits, rec_off, cnt,
                           rec, rec_cap, st, sfirst, slast, max_ents);
        return;
    }
    if (w.nb_u >= 8)
        hipLaunchKernelGGL(k_sync_write_small<8>, dim3(n_spaces), dim3(NT), lds, s, w, flagged, fbits, rec_off, cnt,
                           rec, rec_cap, st, sfirst, slast, max_ents);
    else if (w.nb_u <= 2)
        hipLaunchKernelGGL(k_sync_write_small<2>, dim3(n_spaces), dim3(NT), lds, s, w, flagged, fbits, rec_off, cnt,
                           rec, rec_cap, st, sfirst, slast, max_ents);
    else
        hipLaunchKernelGGL(k_sync_write_small<4>, dim3(n_spaces), dim3(NT), lds, s, w, flagged, fbits, rec_off, cnt,
                           rec, rec_cap, st, sfirst, slast, max_ents);
}

void launch_sync_write(const World& w, const uint32_t* flagged, const uint32_t* fbits, const uint64_t* nf_dev,
                       uint32_t nf_max, const uint64_t* rec_off, const uint32_t* cnt, gw_sync_record* rec,
                       uint64_t rec_cap, DevStats* st, hipStream_t s, uint64_t* pr, float4* pay, bool halves) {
    if (!nf_max) return;
    const dim3 g(std::min(nblk(nf_max, NWAVE), SYNC_MAX_BLOCKS));
    if (halves && !pr) {
        hipLaunchKernelGGL(k_sync_write_h<4>, dim3(std::min(nblk(nf_max, 2 * NWAVE), SYNC_MAX_BLOCKS)), dim3(NT), 0, s,
                           w, flagged, fbits, nf_dev, nf_max, rec_off, cnt, rec, rec_cap, st);
        return;
    }
    if (pr)
        hipLaunchKernelGGL((k_sync_write<4, true>), g, dim3(NT), 0, s, w, flagged, fbits, nf_dev, nf_max, rec_off, cnt,
                           rec, rec_cap, st, pr, pay);
    else if (w.nb_u >= 8)
        hipLaunchKernelGGL(k_sync_write<8>, g, dim3(NT), 0, s, w, flagged, fbits, nf_dev, nf_max, rec_off, cnt, rec,
                           rec_cap, st, pr, pay);
    else if (w.nb_u <= 2)
        hipLaunchKernelGGL(k_sync_write<2>, g, dim3(NT), 0, s, w, flagged, fbits, nf_dev, nf_max, rec_off, cnt, rec,
                           rec_cap, st, pr, pay);
    else
        hipLaunchKernelGGL(k_sync_write<4>, g, dim3(NT), 0, s, w, flagged, fbits, nf_dev, nf_max, rec_off, cnt, rec,
                           rec_cap, st, pr, pay);
}

// ---------------------------------------------------------------------------
// Several gates in use (G = max gate id + 1 <= GATE_DIRECT_MAX): the records
// of each gate form one contiguous partition, in the order of the one-gate
// stream restricted to that gate (entities ascending, the own record first,
// then the neighbours in walk order) -- what a stable sort of the stream by
// gate gives (Entity.go:1208-1219 sends one packet per gate), computed
// without the sort and without a second host sync:
//   count: a lane per flagged entry, counts per (gate, entry) in gate-major
//          cnt[g * nf_max + k]: a mover of this tick's diff from its per-gate
//          split (World.nbg, NBC_GATES); any other entry's window is walked by
//          the whole wave (the watcher's gate from its grid entry);
//   scan:  one exclusive scan over the G * nf_max counts gives every (gate,
//          entry) its first record, and gate g's first record at g * nf_max;
//   write: a wave per entry holds the next position of each gate in lanes
//          0..G-1 and stores each record at its gate's position (ranks inside
//          a chunk from four ballots, the bit planes of the gate ids, whatever
//          G); the gates' first records go to
//          DevStats.gate_base, read with the collect's one host sync.
#ifndef GW_CG_EPW
#define GW_CG_EPW 4
#endif
constexpr int CG_EPW = GW_CG_EPW;   // k_sync_count_g: flagged entries per wave
template <int U>
__global__ void __launch_bounds__(NT) k_sync_count_g(World w, const uint32_t* __restrict__ flagged,
                                                     const uint32_t* __restrict__ fbits, const uint64_t* nf_dev,
                                                     uint32_t nf_max, uint32_t G, uint32_t* __restrict__ cnt) {
    const uint64_t nf = load_n(nf_max, nf_dev);
    const int ln = lane_id();
    const uint64_t stride = (uint64_t)gridDim.x * NWAVE * CG_EPW;
    // a lane per flagged entry, CG_EPW entries per wave: the split of this
    // tick's diff where it has one; the others' windows are then walked one at
    // a time by the whole wave, lane g counting gate g (few entries per wave
    // keep the walks spread over many waves when the split is stale)
    for (uint64_t base = ((uint64_t)blockIdx.x * NWAVE + (threadIdx.x >> 6)) * CG_EPW; base < nf_max; base += stride) {
        const uint64_t k = base + ln;
        const bool mine = ln < CG_EPW && k < nf_max;
        uint32_t e = 0, f = 0, gt = 0;
        AoiEnt a{};
        unsigned long long nc = 0;
        if (mine && k < nf) {
            e = flagged[k];
            f = fbits[k];
            a = w.rec[e].a;
            gt = w.rec[e].gate;
            nc = w.nbc[e];
        }
        bool nbr = false, walk = false;
        if (mine && k < nf && owned_x(w.sp[a.meta & SPACE_MASK], a.x)) {
            if (!(f & GW_SIF_OWN_CLIENT)) gt = 0;            // gt: the own record's gate, 0 for none
            nbr = (f & GW_SIF_NEIGHBOR_CLIENTS) && (a.meta & PRESENT_BIT);
            walk = nbr && !((uint32_t)(nc >> 32) == w.epoch && (nc & NBC_GATES));   // no split from this tick
        } else {
            gt = 0;                                          // (not owned here / past the list: no records)
        }
        if (mine && !walk) {
            unsigned long long sw[4] = {0ull, 0ull, 0ull, 0ull};
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j)
                if (nbr && 4 * j < G) sw[j] = w.nbg[(uint64_t)e * 4 + j];
            cnt[k] = 0;                                      // gate 0 (no client): never a record
#pragma unroll
            for (uint32_t q = 1; q < GATE_DIRECT_MAX; ++q) {
                if (q >= G) break;                           // kernel-uniform
                cnt[(uint64_t)q * nf_max + k] = ((uint32_t)(sw[q >> 2] >> (16 * (q & 3))) & 0xffffu) + (gt == q ? 1u : 0u);
            }
        }
        uint64_t todo = wave_ballot(walk);
        while (todo) {
            const int L = __builtin_ctzll(todo);
            todo &= todo - 1;
            const uint32_t eq = (uint32_t)__builtin_amdgcn_readlane((int)e, L);
            const uint32_t gq = (uint32_t)__builtin_amdgcn_readlane((int)gt, L);
            uint32_t c = (gq && (uint32_t)ln == gq) ? 1u : 0u;   // lane g: records of gate g
            const AoiEnt aq = w.rec[eq].a;
            wave_neighbors_of<U>(w, eq, aq, w.sp[aq.meta & SPACE_MASK], [&](bool rel, uint32_t ws, uint32_t g) {
                // the watcher's gate from its grid entry (ids < 16 here): no gather
                const uint32_t gw = (rel && g != 0) ? (g >> GATE_SHIFT) & 15u : 0u;   // 0: no record
                const uint64_t any = wave_ballot(gw != 0);
                if (!any) return;                         // wave-uniform
                // lane q counts the lanes whose id is q, from the ids' bit planes
                const uint64_t b0 = wave_ballot(gw & 1u), b1 = wave_ballot(gw & 2u);
                const uint64_t b2 = wave_ballot(gw & 4u), b3 = wave_ballot(gw & 8u);
                const uint32_t q = (uint32_t)ln;
                const uint64_t mq = any & ((q & 1u) ? b0 : ~b0) & ((q & 2u) ? b1 : ~b1) & ((q & 4u) ? b2 : ~b2) &
                                    ((q & 8u) ? b3 : ~b3);
                if (q < G) c += (uint32_t)popc64(mq);
            });
            if ((uint32_t)ln < G) cnt[(uint64_t)ln * nf_max + base + L] = c;
        }
    }
}

template <int U>
__global__ void __launch_bounds__(NT) k_sync_write_g(World w, const uint32_t* __restrict__ flagged,
                                                     const uint32_t* __restrict__ fbits, const uint64_t* nf_dev,
                                                     uint32_t nf_max, uint32_t G, const uint64_t* __restrict__ off,
                                                     gw_sync_record* rec, uint64_t rec_cap, DevStats* st) {
    const uint64_t nf = load_n(nf_max, nf_dev);
    const int ln = lane_id();
    const uint64_t lt = lanemask_lt();
    if (st->rec_total > rec_cap) {                        // kernel-uniform: the host grows the buffer, reruns
        if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(&st->overflow, 1ull);
        return;
    }
    if (blockIdx.x == 0 && threadIdx.x < G) st->gate_base[threadIdx.x] = off[(uint64_t)threadIdx.x * nf_max];
    const uint64_t stride = (uint64_t)gridDim.x * NWAVE;
    for (uint64_t k = (uint64_t)blockIdx.x * NWAVE + (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
         k < nf; k += stride) {
        const uint32_t e = flagged[k], f = fbits[k];
        const AoiEnt a = w.rec[e].a;
        const uint32_t gt = w.rec[e].gate;
        const SpaceP P = w.sp[a.meta & SPACE_MASK];
        if (!owned_x(P, a.x)) continue;
        const float4 p = w.rec[e].p;
        uint64_t at = (uint32_t)ln < G ? off[(uint64_t)ln * nf_max + k] : 0ull;   // lane g: gate g's next record
        if ((f & GW_SIF_OWN_CLIENT) && gt) {
            const uint64_t o = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(at >> 32), (int)gt) << 32) |
                               (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)at, (int)gt);
            if (ln == 0) st_record_nt(rec + o, e, e, p);
            if ((uint32_t)ln == gt) ++at;
        }
        if (!(f & GW_SIF_NEIGHBOR_CLIENTS) || !(a.meta & PRESENT_BIT)) continue;
        wave_neighbors_of<U>(w, e, a, P, [&](bool rel, uint32_t ws, uint32_t g) {
            const uint32_t gw = (rel && g != 0) ? (g >> GATE_SHIFT) & 15u : 0u;   // (grid entry: no gather)
            const uint64_t any = wave_ballot(gw != 0);
            if (!any) return;                             // wave-uniform
            // the lanes of each gate from the gate ids' four bit planes (one
            // ballot each, whatever G): lanes_of(q) = the lanes whose id is q
            const uint64_t b0 = wave_ballot(gw & 1u), b1 = wave_ballot(gw & 2u);
            const uint64_t b2 = wave_ballot(gw & 4u), b3 = wave_ballot(gw & 8u);
            auto lanes_of = [&](uint32_t q) {
                return any & ((q & 1u) ? b0 : ~b0) & ((q & 2u) ? b1 : ~b1) & ((q & 4u) ? b2 : ~b2) &
                       ((q & 8u) ? b3 : ~b3);
            };
            // my gate's next position sits in lane gw
            const uint32_t olo = (uint32_t)__shfl((int)(uint32_t)at, (int)gw, 64);
            const uint32_t ohi = (uint32_t)__shfl((int)(uint32_t)(at >> 32), (int)gw, 64);
            const uint64_t pos = (((uint64_t)ohi << 32) | olo) + (uint64_t)popc64(lanes_of(gw) & lt);
            if ((uint32_t)ln < G) at += (uint64_t)popc64(lanes_of((uint32_t)ln));   // lane 0: none (any excludes id 0)
            if (gw != 0) st_record_nt(rec + pos, ws, e, p);
        });
    }
}

void launch_sync_gates(const World& w, const uint32_t* flagged, const uint32_t* fbits, const uint64_t* nf_dev,
                       uint32_t nf_max, uint32_t G, uint32_t* cnt, hipStream_t s) {
    if (!nf_max) return;
    const dim3 g(std::min(nblk(nf_max, NWAVE * CG_EPW), SYNC_MAX_BLOCKS));   // CG_EPW entries per wave
    hipLaunchKernelGGL(k_sync_count_g<4>, g, dim3(NT), 0, s, w, flagged, fbits, nf_dev, nf_max, G, cnt);
}
void launch_sync_write_gates(const World& w, const uint32_t* flagged, const uint32_t* fbits, const uint64_t* nf_dev,
                             uint32_t nf_max, uint32_t G, const uint64_t* off, gw_sync_record* rec, uint64_t rec_cap,
                             DevStats* st, hipStream_t s) {
    if (!nf_max) return;
    const dim3 g(std::min(nblk(nf_max, NWAVE), SYNC_MAX_BLOCKS));
    hipLaunchKernelGGL(k_sync_write_g<4>, g, dim3(NT), 0, s, w, flagged, fbits, nf_dev, nf_max, G, off, rec, rec_cap,
                       st);
}

// 24-B records from sorted (watcher, entity) pairs (through idx, the gate
// grouping's permutation, when given; the entity's payload from its slot)
// and, in the same pass, the client segment table of the stream (what
// k_client_heads + scan + k_client_segments derive from written records):
// a head per first record of a watcher, compacted by a
// decoupled look-back (prim.hpp) into client_slot / client_off; the
// watchers come from the sorted keys, not from a re-read of the records.
// Tiles of SCAN_TILE pairs, striped: lane l's predecessor is lane l-1's
// element, lane 0 loads its own.
__global__ void __launch_bounds__(NT) k_records_seg(World w, const uint64_t* __restrict__ pr,
                                                    const uint32_t* __restrict__ idx,
                                                    const uint32_t* __restrict__ flagged,
                                                    const float4* __restrict__ pay, uint64_t n,
                                                    gw_sync_record* __restrict__ out,
                                                    uint32_t* __restrict__ client_slot,
                                                    uint64_t* __restrict__ client_off, uint32_t* n_clients,
                                                    unsigned long long* __restrict__ status,
                                                    unsigned long long* __restrict__ ticket, unsigned long long tbase,
                                                    uint32_t tag) {
    constexpr int IPT = SCAN_IPT;
    constexpr int G = 4;                                 // rows whose gathers are in flight together
    __shared__ uint32_t lds[IPT * NWAVE];
    __shared__ uint32_t s_tile, s_prefix;
    __shared__ unsigned long long stg[NWAVE][3 * 64];     // a wave's 64 records, written out coalesced
    if (threadIdx.x == 0) s_tile = (uint32_t)(atomicAdd(ticket, 1ull) - tbase);
    __syncthreads();
    const uint32_t tile = s_tile;
    const uint64_t t0 = (uint64_t)tile * (IPT * NT);
    const int ln = lane_id();
    unsigned long long* sb = stg[threadIdx.x >> 6];
    uint32_t wt[IPT], c[IPT];
#pragma unroll
    for (int j0 = 0; j0 < IPT; j0 += G) {
        uint32_t e[G], pw[G], f[G];
        float4 p[G];
#pragma unroll
        for (int u = 0; u < G; ++u) {
            const uint64_t i = t0 + (uint64_t)(j0 + u) * NT + threadIdx.x;
            const uint32_t q = i < n ? (idx ? idx[i] : (uint32_t)i) : 0u;
            const uint64_t x = i < n ? pr[q] : ~0ull;
            wt[j0 + u] = (uint32_t)x;
            f[u] = (uint32_t)(x >> 32);
            pw[u] = (ln == 0 && i < n && i > 0) ? (uint32_t)pr[idx ? idx[i - 1] : (uint32_t)(i - 1)] : 0xffffffffu;
        }
#pragma unroll
        for (int u = 0; u < G; ++u) {                    // the flagged entity's slot and payload
            const uint64_t i = t0 + (uint64_t)(j0 + u) * NT + threadIdx.x;
            if (i < n) {
                e[u] = flagged[f[u]];
                p[u] = pay[f[u]];
            }
        }
#pragma unroll
        for (int u = 0; u < G; ++u) {
            const uint64_t i = t0 + (uint64_t)(j0 + u) * NT + threadIdx.x;
            uint32_t prev = (uint32_t)__shfl_up((int)wt[j0 + u], 1, 64);
            if (ln == 0) prev = pw[u];
            c[j0 + u] = (i < n && (i == 0 || prev != wt[j0 + u])) ? 1u : 0u;
            // the row's 64 records (1536 B) staged, then 3 x 64 contiguous 8-B
            // stores (one 24-B record per lane as three strided stores leaves
            // partial lines behind each instruction)
            if (i < n) {
                sb[3 * ln] = ((unsigned long long)e[u] << 32) | wt[j0 + u];
                sb[3 * ln + 1] = ((unsigned long long)__float_as_uint(p[u].y) << 32) | __float_as_uint(p[u].x);
                sb[3 * ln + 2] = ((unsigned long long)__float_as_uint(p[u].w) << 32) | __float_as_uint(p[u].z);
            }
            wave_sync();
            const uint64_t ib = i - (uint64_t)ln;                 // the wave's first record of the row
            if (ib < n) {
                const uint32_t words = 3u * (uint32_t)min<uint64_t>(64, n - ib);
                unsigned long long* dst = reinterpret_cast<unsigned long long*>(out + ib);
#pragma unroll
                for (uint32_t q = 0; q < 3; ++q) {
                    const uint32_t x = q * 64 + (uint32_t)ln;
                    if (x < words) __builtin_nontemporal_store(sb[x], dst + x);
                }
            }
            wave_sync();
        }
    }
    uint32_t head = 0;
#pragma unroll
    for (int j = 0; j < IPT; ++j) head |= c[j] << j;
    uint32_t tot;
    tile_excl_scan_striped<uint32_t, IPT>(c, lds, tot);
    if (threadIdx.x < 64) {
        const uint32_t excl = scan_lookback<uint32_t>(status, tile, tag, tot);
        if (threadIdx.x == 0) s_prefix = excl;
    }
    __syncthreads();
    const uint32_t pre = s_prefix;
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        if ((head >> j) & 1u) {
            const uint32_t at = pre + c[j];
            client_slot[at] = wt[j];
            client_off[at] = t0 + (uint64_t)j * NT + threadIdx.x;
        }
    }
    if (tile == gridDim.x - 1 && threadIdx.x == 0) {
        *n_clients = pre + tot;
        client_off[pre + tot] = n;                       // end of the last client
    }
}
void launch_records_seg(const World& w, const uint64_t* pairs, const uint32_t* idx, const uint32_t* flagged, const float4* pay, uint64_t n, gw_sync_record* out,
                        uint32_t* client_slot, uint64_t* client_off, uint32_t* n_clients, ScanCtx& sc,
                        hipStream_t s) {
    if (!n) return;
    const uint32_t nb = (uint32_t)((n + SCAN_TILE - 1) / SCAN_TILE);
    if (sc.tag >= SCAN_TAG_MAX) {
        (void)hipMemsetAsync(sc.status, 0, sc.max_tiles * SCAN_WORDS * 8, s);
        sc.tag = 0;
    }
    ++sc.tag;
    hipLaunchKernelGGL(k_records_seg, dim3(nb), dim3(NT), 0, s, w, pairs, idx, flagged, pay, n, out, client_slot,
                       client_off, n_clients, sc.status, sc.ticket, sc.tbase, sc.tag);
    sc.tbase += nb;
}

// per-gate record histogram: LDS buckets for gates < 256, global atomics above
__global__ void __launch_bounds__(NT) k_gate_hist(const gw_sync_record* __restrict__ rec, const uint64_t* n_dev,
                                                  uint64_t n_max, const uint16_t* __restrict__ gate, uint32_t* hist) {
    __shared__ uint32_t h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    uint64_t n = load_n(n_max, n_dev);
    for (uint64_t r = (uint64_t)blockIdx.x * NT + threadIdx.x; r < n; r += (uint64_t)gridDim.x * NT) {
        uint32_t g = gate[rec[r].watcher];
        if (g < 256) atomicAdd(&h[g], 1u); else atomicAdd(&hist[g], 1u);
    }
    __syncthreads();
    if (h[threadIdx.x]) atomicAdd(&hist[threadIdx.x], h[threadIdx.x]);
}
void launch_gate_hist(const gw_sync_record* rec, const uint64_t* n_dev, uint64_t n_max, const uint16_t* gate,
                      uint32_t* hist, hipStream_t s) {
    uint32_t nb = nblk1(n_max, NT * 16);
    if (nb > 2048) nb = 2048;
    hipLaunchKernelGGL(k_gate_hist, dim3(nb), dim3(NT), 0, s, rec, n_dev, n_max, gate, hist);
}
__global__ void __launch_bounds__(NT) k_gate_keys(const gw_sync_record* __restrict__ rec, const uint64_t* n_dev,
                                                  uint64_t n_max, const uint16_t* __restrict__ gate, uint32_t* keys,
                                                  uint32_t* vals) {
    uint64_t n = load_n(n_max, n_dev);
    uint64_t r = (uint64_t)blockIdx.x * NT + threadIdx.x;
    if (r >= n) return;
    keys[r] = gate[rec[r].watcher];
    vals[r] = (uint32_t)r;
}
void launch_gate_keys(const gw_sync_record* rec, const uint64_t* n_dev, uint64_t n_max, const uint16_t* gate,
                      uint32_t* keys, uint32_t* vals, hipStream_t s) {
    if (!n_max) return;
    hipLaunchKernelGGL(k_gate_keys, dim3(nblk(n_max, NT)), dim3(NT), 0, s, rec, n_dev, n_max, gate, keys, vals);
}
__global__ void __launch_bounds__(NT) k_gather_records(const gw_sync_record* __restrict__ in,
                                                       const uint32_t* __restrict__ idx, const uint64_t* n_dev,
                                                       uint64_t n_max, gw_sync_record* out) {
    uint64_t n = load_n(n_max, n_dev);
    uint64_t r = (uint64_t)blockIdx.x * NT + threadIdx.x;
    if (r < n) out[r] = in[idx[r]];
}
// ---------------------------------------------------------------------------
// Per-client grouping of the record stream (GateService.handleSyncPositionYaw
// OnClients, GateService.go:350-375, done on the device): the keys of a stable
// sort by watcher, then the client segments of the sorted stream (a flag per
// first record of a watcher, scanned, compacted into slot + offset).
__global__ void __launch_bounds__(NT) k_watcher_keys(const gw_sync_record* __restrict__ rec, uint64_t n,
                                                     uint32_t* keys, uint32_t* vals) {
    const uint64_t r = (uint64_t)blockIdx.x * NT + threadIdx.x;
    if (r >= n) return;
    keys[r] = rec[r].watcher;
    vals[r] = (uint32_t)r;
}
void launch_watcher_keys(const gw_sync_record* rec, uint64_t n, uint32_t* keys, uint32_t* vals, hipStream_t s) {
    if (!n) return;
    hipLaunchKernelGGL(k_watcher_keys, dim3(nblk(n, NT)), dim3(NT), 0, s, rec, n, keys, vals);
}
__global__ void __launch_bounds__(NT) k_client_heads(const gw_sync_record* __restrict__ rec, uint64_t n,
                                                     uint32_t* head) {
    const uint64_t r = (uint64_t)blockIdx.x * NT + threadIdx.x;
    if (r >= n) return;
    head[r] = (r == 0 || rec[r].watcher != rec[r - 1].watcher) ? 1u : 0u;
}
__global__ void __launch_bounds__(NT) k_client_segments(const gw_sync_record* __restrict__ rec, uint64_t n,
                                                        const uint32_t* __restrict__ head,
                                                        const uint32_t* __restrict__ pos, uint32_t* client_slot,
                                                        uint64_t* client_off) {
    const uint64_t r = (uint64_t)blockIdx.x * NT + threadIdx.x;
    if (r >= n) return;
    if (head[r]) {
        client_slot[pos[r]] = rec[r].watcher;
        client_off[pos[r]] = r;
    }
    if (r == n - 1) client_off[pos[r] + head[r]] = n;    // end of the last client
}
void launch_client_segments(const gw_sync_record* rec, uint64_t n, uint32_t* head, uint32_t* pos,
                            uint32_t* n_clients, uint32_t* client_slot, uint64_t* client_off, ScanCtx& sc,
                            hipStream_t s) {
    if (!n) return;
    hipLaunchKernelGGL(k_client_heads, dim3(nblk(n, NT)), dim3(NT), 0, s, rec, n, head);
    scan_exclusive<uint32_t, uint32_t>(head, pos, n, nullptr, sc, n_clients, s);
    hipLaunchKernelGGL(k_client_segments, dim3(nblk(n, NT)), dim3(NT), 0, s, rec, n, head, pos, client_slot,
                       client_off);
}

void launch_gather_records(const gw_sync_record* in, const uint32_t* idx, const uint64_t* n_dev, uint64_t n_max,
                           gw_sync_record* out, hipStream_t s) {
    if (!n_max) return;
    hipLaunchKernelGGL(k_gather_records, dim3(nblk(n_max, NT)), dim3(NT), 0, s, in, idx, n_dev, n_max, out);
}

// ---------------------------------------------------------------------------
// client attach / detach (GameClient.go:14-27): the gate copy in the grid entry
// is patched too, so a collect after set_clients sees the new gates
// gate[] (and its copy in the slot record) always; the CLIENT_BIT of the slot's grid entry only while the grid
// is current (grid_ok: a rebuild takes the bits from gate[] anyway, and gidx
// of slots entered since the last build is not valid)
__global__ void __launch_bounds__(NT) k_set_clients(World w, const uint32_t* slots, const uint16_t* gates,
                                                    uint32_t n, int grid_ok) {
    uint32_t i = blockIdx.x * NT + threadIdx.x;
    if (i >= n || slots[i] >= w.cap) return;
    const uint32_t s = slots[i];
    w.gate[s] = gates[i];
    w.rec[s].gate = gates[i];
    const AoiEnt a = w.rec[s].a;
    if (grid_ok && (a.meta & PRESENT_BIT)) {
        const uint32_t k = w.gn_start[cell_of(w.sp[a.meta & SPACE_MASK], a.x, a.z)] + w.rec[s].gidx;
        if (k < w.cap) {
            GEnt* g = w.gn + k;
            if (g->slot == s) g->meta = (g->meta & ~(CLIENT_BIT | GATE_MASK)) | gate_meta(gates[i]);
        }
    }
}
void launch_set_clients(const World& w, const uint32_t* slots, const uint16_t* gates, uint32_t n, bool grid_ok,
                        hipStream_t s) {
    if (!n) return;
    hipLaunchKernelGGL(k_set_clients, dim3(nblk(n, NT)), dim3(NT), 0, s, w, slots, gates, n, grid_ok ? 1 : 0);
}

// InterestedIn(slot) (== InterestedBy): related slots, unordered
__global__ void __launch_bounds__(64) k_neighbors(World w, uint32_t slot, uint32_t* out, uint32_t* n_out,
                                                  uint32_t cap) {
    const uint64_t lt = lanemask_lt();
    uint32_t n = 0;
    wave_neighbors(w, slot, [&](bool rel, uint32_t ws, uint32_t) {
        const uint64_t bt = wave_ballot(rel);
        const uint32_t i = n + (uint32_t)popc64(bt & lt);
        if (rel && i < cap) out[i] = ws;
        n += (uint32_t)popc64(bt);
    });
    if (lane_id() == 0) *n_out = n;
}
void launch_neighbors(const World& w, uint32_t slot, uint32_t* out, uint32_t* n_out, uint32_t cap, hipStream_t s) {
    hipLaunchKernelGGL(k_neighbors, dim3(1), dim3(64), 0, s, w, slot, out, n_out, cap);
}

// sum of |InterestedIn| over all present entities (one wave per entity)
__global__ void __launch_bounds__(NT) k_count_all(World w, uint64_t np, unsigned long long* total) {
    const uint64_t i = (uint64_t)blockIdx.x * NWAVE + (threadIdx.x >> 6);
    if (i >= np) return;
    uint32_t n = 0;
    wave_neighbors(w, w.gn[i].slot, [&](bool rel, uint32_t, uint32_t) { n += (uint32_t)popc64(wave_ballot(rel)); });
    if (lane_id() == 0 && n) atomicAdd(total, (unsigned long long)n);
}
void launch_count_all(const World& w, uint64_t n_present, unsigned long long* total, hipStream_t s) {
    if (n_present) hipLaunchKernelGGL(k_count_all, dim3(nblk(n_present, NWAVE)), dim3(NT), 0, s, w, n_present, total);
}

__global__ void k_fill_u32(uint32_t* p, uint32_t v, uint64_t n) {
    uint64_t i = (uint64_t)blockIdx.x * NT + threadIdx.x;
    if (i < n) p[i] = v;
}
__global__ void k_fill_i32(int32_t* p, int32_t v, uint64_t n) {
    uint64_t i = (uint64_t)blockIdx.x * NT + threadIdx.x;
    if (i < n) p[i] = v;
}
void launch_fill_u32(uint32_t* p, uint32_t v, uint64_t n, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_fill_u32, dim3(nblk(n, NT)), dim3(NT), 0, s, p, v, n);
}
void launch_fill_i32(int32_t* p, int32_t v, uint64_t n, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_fill_i32, dim3(nblk(n, NT)), dim3(NT), 0, s, p, v, n);
}

// ---------------------------------------------------------------------------
// Client messages.  Records are runs of W u32 words
// whose first word is the receiving watcher slot.
//
// (a) AOI events -> client messages: Entity.interest / uninterest call
// e.client.sendCreateEntity(other) / sendDestroyEntity(other), a no-op when the
// watcher has no client (Entity.go:236-246, GameClient.go:37-59).  One pass
// per kind: a tile of SCAN_TILE canonical events (striped) flags the events
// whose watcher has a client, takes its offset by a decoupled look-back
// (prim.hpp) and writes its messages in the (watcher, target) order; creates
// carry the target's position and yaw (GameClient.go:49-52).  The last tile
// writes the count.
__global__ void __launch_bounds__(NT) k_event_client_compact(const gw_event* __restrict__ ev, uint64_t n,
                                                             const uint16_t* __restrict__ gate,
                                                             const SlotRec* __restrict__ srec, uint32_t* out,
                                                             int create, uint32_t* n_out,
                                                             unsigned long long* __restrict__ status,
                                                             unsigned long long* __restrict__ ticket,
                                                             unsigned long long tbase, uint32_t tag) {
    constexpr int IPT = SCAN_IPT;
    __shared__ uint32_t lds[IPT * NWAVE];
    __shared__ uint32_t s_tile, s_prefix;
    if (threadIdx.x == 0) s_tile = (uint32_t)(atomicAdd(ticket, 1ull) - tbase);
    __syncthreads();
    const uint32_t tile = s_tile;
    const uint64_t t0 = (uint64_t)tile * (IPT * NT);
    gw_event e[IPT];
    uint32_t c[IPT];
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        const uint64_t i = t0 + (uint64_t)j * NT + threadIdx.x;
        e[j].watcher = 0;
        e[j].target = 0;
        if (i < n) e[j] = ev[i];
    }
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        const uint64_t i = t0 + (uint64_t)j * NT + threadIdx.x;
        c[j] = (i < n && gate[e[j].watcher] != 0) ? 1u : 0u;
    }
    uint32_t flag = 0;
#pragma unroll
    for (int j = 0; j < IPT; ++j) flag |= c[j] << j;
    uint32_t tot;
    tile_excl_scan_striped<uint32_t, IPT>(c, lds, tot);
    if (threadIdx.x < 64) {
        const uint32_t excl = scan_lookback<uint32_t>(status, tile, tag, tot);
        if (threadIdx.x == 0) s_prefix = excl;
    }
    __syncthreads();
    const uint32_t pre = s_prefix;
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        if (!((flag >> j) & 1u)) continue;
        const uint32_t at = pre + c[j];
        if (create) {
            const float4 p = srec[e[j].target].p;
            gw_sync_record m;
            m.watcher = e[j].watcher; m.entity = e[j].target; m.x = p.x; m.y = p.y; m.z = p.z; m.yaw = p.w;
            ((gw_sync_record*)out)[at] = m;
        } else {
            ((gw_event*)out)[at] = e[j];
        }
    }
    if (tile == gridDim.x - 1 && threadIdx.x == 0) *n_out = pre + tot;
}
void launch_event_client_compact(const gw_event* ev, uint64_t n, const uint16_t* gate, const SlotRec* rec,
                                 uint32_t* out, bool create, uint32_t* n_out, ScanCtx& sc, hipStream_t s) {
    if (!n) return;
    const uint32_t nb = (uint32_t)((n + SCAN_TILE - 1) / SCAN_TILE);
    if (sc.tag >= SCAN_TAG_MAX) {
        (void)hipMemsetAsync(sc.status, 0, sc.max_tiles * SCAN_WORDS * 8, s);
        sc.tag = 0;
    }
    ++sc.tag;
    hipLaunchKernelGGL(k_event_client_compact, dim3(nb), dim3(NT), 0, s, ev, n, gate, rec, out, create ? 1 : 0,
                       n_out, sc.status, sc.ticket, sc.tbase, sc.tag);
    sc.tbase += nb;
}

// (b) AllClients fan-out: CallAllClients and every AllClients attribute
// notification send to e.client, then to n.client for n in e.InterestedBy
// (Entity.go:743-749, 814-917).  Item k (entity items[k]) -> deliveries
// (watcher, k): the own one first, then the related entities with a client,
// from the current grid (one wave per item, like the collect).  A delivery is
// two u32 words, the sort key and its value: the entity is items[k], so the
// 12-B record is built once, after the sort (k_fanout_final).
// Counts: a lane per item takes the diff's cached count of neighbours with a
// client when this epoch's tick made it (a call on a mover of the last tick),
// the rest are walked one at a time by the wave (as k_sync_count).
template <int U>
__global__ void __launch_bounds__(NT) k_fanout_count(World w, const uint32_t* __restrict__ items, uint32_t n,
                                                     uint32_t* cnt) {
    const int ln = lane_id();
    const uint64_t stride = (uint64_t)gridDim.x * NT;
    for (uint64_t base = (uint64_t)blockIdx.x * NT + (threadIdx.x & ~63u); base < n; base += stride) {
        const uint64_t k = base + ln;
        const bool valid = k < n;
        uint32_t e = 0, r = 0;
        bool walk = false;
        if (valid) {
            e = items[k];
            const AoiEnt a = w.rec[e].a;
            const uint32_t g = w.rec[e].gate;
            const unsigned long long c = w.nbc[e];
            r = g ? 1u : 0u;
            if (a.meta & PRESENT_BIT) {
                if ((uint32_t)(c >> 32) == w.epoch) r += (uint32_t)c & NBC_COUNT;
                else walk = true;
            }
        }
        uint64_t todo = wave_ballot(walk);
        while (todo) {
            const int q = __builtin_ctzll(todo);
            todo &= todo - 1;
            const uint32_t eq = (uint32_t)__builtin_amdgcn_readlane((int)e, q);
            uint32_t m = 0;
            wave_neighbors<U>(w, eq, [&](bool rel, uint32_t, uint32_t g) {
                m += (uint32_t)popc64(wave_ballot(rel && g != 0));
            });
            if (ln == q) r += m;
        }
        if (valid) cnt[k] = r;
    }
}
template <int U>
__global__ void __launch_bounds__(NT) k_fanout_write(World w, const uint32_t* __restrict__ items, uint32_t n,
                                                     const uint64_t* __restrict__ off, uint64_t* __restrict__ pr) {
    const uint64_t lt = lanemask_lt();
    const uint64_t stride = (uint64_t)gridDim.x * NWAVE;
    for (uint64_t k = (uint64_t)blockIdx.x * NWAVE + (threadIdx.x >> 6); k < n; k += stride) {
        const uint32_t e = items[k];
        uint64_t at = off[k];
        if (w.gate[e]) {
            if (lane_id() == 0) pr[at] = (k << 32) | e;
            ++at;
        }
        wave_neighbors<U>(w, e, [&](bool rel, uint32_t ws, uint32_t g) {
            const bool take = rel && g != 0;
            const uint64_t bt = wave_ballot(take);
            if (take) pr[at + (uint64_t)popc64(bt & lt)] = (k << 32) | ws;
            at += (uint64_t)popc64(bt);
        });
    }
}
void launch_fanout(const World& w, const uint32_t* items, uint32_t n, uint32_t* cnt, const uint64_t* off,
                   uint64_t* pairs, hipStream_t s) {
    if (!n) return;
    if (cnt)
        hipLaunchKernelGGL(k_fanout_count<4>, dim3(std::min(nblk(n, NT), SYNC_MAX_BLOCKS)), dim3(NT), 0, s, w, items,
                           n, cnt);
    else
        hipLaunchKernelGGL(k_fanout_write<4>, dim3(std::min(nblk(n, NWAVE), SYNC_MAX_BLOCKS)), dim3(NT), 0, s, w,
                           items, n, off, pairs);
}
// the records from the sorted (watcher, item) pairs, through idx (the gate
// grouping's permutation) when given; gate keys of the pairs for that grouping
__global__ void __launch_bounds__(NT) k_fanout_final(const uint64_t* __restrict__ pr,
                                                     const uint32_t* __restrict__ idx,
                                                     const uint32_t* __restrict__ items, uint64_t n,
                                                     gw_fanout_rec* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * NT + threadIdx.x;
    if (i >= n) return;
    const uint32_t j = idx ? idx[i] : (uint32_t)i;
    const uint64_t x = pr[j];
    gw_fanout_rec r;
    r.watcher = (uint32_t)x;
    r.item = (uint32_t)(x >> 32);
    r.entity = items[r.item];
    out[i] = r;
}
__global__ void __launch_bounds__(NT) k_gate_keys(const uint64_t* __restrict__ pr, const uint16_t* __restrict__ gate,
                                                  uint64_t n, uint32_t* keys, uint32_t* vals, uint32_t* hist) {
    __shared__ uint32_t h[NT];
    h[threadIdx.x] = 0;
    __syncthreads();
    for (uint64_t i = (uint64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (uint64_t)gridDim.x * NT) {
        const uint32_t g = gate[(uint32_t)pr[i]];
        keys[i] = g;
        vals[i] = (uint32_t)i;
        if (g < NT) atomicAdd(&h[g], 1u); else atomicAdd(&hist[g], 1u);
    }
    __syncthreads();
    if (h[threadIdx.x]) atomicAdd(&hist[threadIdx.x], h[threadIdx.x]);
}
void launch_fanout_final(const uint64_t* pairs, const uint32_t* idx, const uint32_t* items, uint64_t n,
                         gw_fanout_rec* out, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_fanout_final, dim3(nblk(n, NT)), dim3(NT), 0, s, pairs, idx, items, n, out);
}
void launch_gate_keys(const uint64_t* pairs, const uint16_t* gate, uint64_t n, uint32_t* keys, uint32_t* vals,
                      uint32_t* hist, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_gate_keys, dim3(std::min<uint32_t>(nblk(n, NT), 2048)), dim3(NT), 0, s, pairs, gate,
                              n, keys, vals, hist);
}

// (c) stable grouping of a message stream: keys (watcher, or gate(watcher)),
// gather of W-word records by the sorted indices (one thread per output word)
template <int W>
__global__ void __launch_bounds__(NT) k_msg_keys(const uint32_t* __restrict__ rec, uint64_t n,
                                                 const uint16_t* __restrict__ gate, uint32_t* keys, uint32_t* vals) {
    const uint64_t r = (uint64_t)blockIdx.x * NT + threadIdx.x;
    if (r >= n) return;
    const uint32_t w = rec[r * W];
    keys[r] = gate ? (uint32_t)gate[w] : w;
    vals[r] = (uint32_t)r;
}
template <int W>
__global__ void __launch_bounds__(NT) k_msg_gate_hist(const uint32_t* __restrict__ rec, uint64_t n,
                                                      const uint16_t* __restrict__ gate, uint32_t* hist) {
    __shared__ uint32_t h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    for (uint64_t r = (uint64_t)blockIdx.x * NT + threadIdx.x; r < n; r += (uint64_t)gridDim.x * NT) {
        const uint32_t g = gate[rec[r * W]];
        if (g < 256) atomicAdd(&h[g], 1u); else atomicAdd(&hist[g], 1u);
    }
    __syncthreads();
    if (h[threadIdx.x]) atomicAdd(&hist[threadIdx.x], h[threadIdx.x]);
}
template <int W>
__global__ void __launch_bounds__(NT) k_msg_gather(const uint32_t* __restrict__ in, const uint32_t* __restrict__ idx,
                                                   uint64_t n, uint32_t* out) {
    const uint64_t t = (uint64_t)blockIdx.x * NT + threadIdx.x;
    if (t >= n * W) return;
    const uint64_t r = t / W;
    out[t] = in[(uint64_t)idx[r] * W + (t - r * W)];
}
#define GW_MSG_W(words, stmt)                      \
    switch (words) {                               \
    case 2: { constexpr int W = 2; stmt; } break;  \
    case 3: { constexpr int W = 3; stmt; } break;  \
    default: { constexpr int W = 6; stmt; } break; \
    }
void launch_msg_keys(const uint32_t* rec, int words, uint64_t n, const uint16_t* gate, uint32_t* keys, uint32_t* vals,
                     hipStream_t s) {
    if (!n) return;
    GW_MSG_W(words, hipLaunchKernelGGL(k_msg_keys<W>, dim3(nblk(n, NT)), dim3(NT), 0, s, rec, n, gate, keys, vals));
}
void launch_msg_gate_hist(const uint32_t* rec, int words, uint64_t n, const uint16_t* gate, uint32_t* hist,
                          hipStream_t s) {
    if (!n) return;
    uint32_t nb = nblk1(n, NT * 16);
    if (nb > 2048) nb = 2048;
    GW_MSG_W(words, hipLaunchKernelGGL(k_msg_gate_hist<W>, dim3(nb), dim3(NT), 0, s, rec, n, gate, hist));
}
void launch_msg_gather(const uint32_t* in, int words, const uint32_t* idx, uint64_t n, uint32_t* out,
                       hipStream_t s) {
    if (!n) return;
    GW_MSG_W(words, hipLaunchKernelGGL(k_msg_gather<W>, dim3(nblk(n * W, NT)), dim3(NT), 0, s, in, idx, n, out));
}
#undef GW_MSG_W

// ---------------------------------------------------------------------------
// ids (16-B values per slot) and the game->gate wire encode (Entity.go:
// 1210-1266): per gate with records, u16 1502, u16 gateid, then 48-B records
// clientid(watcher) eid(entity) f32 x y z yaw, all little-endian.  One thread
// per output dword (coalesced stores): record r's packet by a binary search
// over the packets' first records, dword j of the record from the client id
// (j < 4), the entity id (j < 8) or the payload.
__global__ void __launch_bounds__(NT) k_put16(uint4* table, const uint32_t* __restrict__ slots,
                                              const uint4* __restrict__ vals, uint32_t n) {
    const uint32_t i = blockIdx.x * NT + threadIdx.x;
    if (i < n) table[slots[i]] = vals[i];
}
void launch_put16(uint4* table, const uint32_t* slots, const uint4* vals, uint32_t n, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_put16, dim3(nblk(n, NT)), dim3(NT), 0, s, table, slots, vals, n);
}
__global__ void __launch_bounds__(NT) k_wire_encode(const gw_sync_record* __restrict__ rec, uint64_t R,
                                                    const WirePacket* __restrict__ pk, uint32_t npk,
                                                    const uint4* __restrict__ eid, const uint4* __restrict__ cid,
                                                    uint32_t* __restrict__ out) {
    const uint64_t t = (uint64_t)blockIdx.x * NT + threadIdx.x;
    if (t < npk) out[pk[t].byte_off / 4] = 1502u | (pk[t].gate << 16);   // packet headers
    const uint64_t r = t / 12;
    if (r >= R) return;
    const uint32_t j = (uint32_t)(t - r * 12);
    uint32_t lo = 0, hi = npk;                               // last packet with rec0 <= r
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (pk[mid].rec0 <= r) lo = mid; else hi = mid;
    }
    const WirePacket p = pk[lo];
    const gw_sync_record e = rec[r];
    uint32_t v;
    if (j < 4) {
        const uint4 c = cid[e.watcher];
        v = j == 0 ? c.x : j == 1 ? c.y : j == 2 ? c.z : c.w;
    } else if (j < 8) {
        const uint4 c = eid[e.entity];
        v = j == 4 ? c.x : j == 5 ? c.y : j == 6 ? c.z : c.w;
    } else {
        const float f = j == 8 ? e.x : j == 9 ? e.y : j == 10 ? e.z : e.yaw;
        v = __float_as_uint(f);
    }
    out[(p.byte_off + 4) / 4 + (r - p.rec0) * 12 + j] = v;
}
void launch_wire_encode(const gw_sync_record* rec, uint64_t R, const WirePacket* pk, uint32_t npk,
                        const uint4* eid, const uint4* cid, uint32_t* out, hipStream_t s) {
    const uint64_t threads = std::max<uint64_t>(R * 12, npk);
    if (threads) hipLaunchKernelGGL(k_wire_encode, dim3(nblk(threads, NT)), dim3(NT), 0, s, rec, R, pk, npk, eid, cid, out);
}

// ---------------------------------------------------------------------------
// primitive instantiations for the host code
uint64_t radix_tile() { return RS_TILE; }
uint64_t radix2_tile() { return RS2_TILE; }
uint64_t radix2_scratch(uint64_t n_max) { return radix2_scratch_words(n_max); }
uint64_t scan_tile() { return SCAN_TILE; }
uint64_t scan_words() { return SCAN_WORDS; }
void scan_u32_u32(const uint32_t* in, uint32_t* out, uint64_t n_max, const uint64_t* n_dev, ScanCtx& sc,
                  uint32_t* total, hipStream_t s) {
    scan_exclusive<uint32_t, uint32_t>(in, out, n_max, n_dev, sc, total, s);
}
void scan_u32_u64(const uint32_t* in, uint64_t* out, uint64_t n_max, const uint64_t* n_dev, ScanCtx& sc,
                  uint64_t* total, hipStream_t s) {
    scan_exclusive<uint32_t, uint64_t>(in, out, n_max, n_dev, sc, total, s);
}
void scan_u64_u64(const uint64_t* in, uint64_t* out, uint64_t n_max, const uint64_t* n_dev, ScanCtx& sc,
                  uint64_t* total, hipStream_t s) {
    scan_exclusive<uint64_t, uint64_t>(in, out, n_max, n_dev, sc, total, s);
}
int sort_pairs64(uint64_t* p0, uint64_t* p1, uint64_t n_max, const uint64_t* n_dev, int lo_bit, int hi_bit,
                 RadixTmp& tmp, hipStream_t s) {
    return radix_sort2_p64(p0, p1, n_max, n_dev, lo_bit, hi_bit, tmp.os, s);
}
int sort_u32_u32(uint32_t* k0, uint32_t* v0, uint32_t* k1, uint32_t* v1, uint64_t n_max, const uint64_t* n_dev,
                 int lo_bit, int hi_bit, RadixTmp& tmp, hipStream_t s) {
    // the pairs of the client paths (fanout, per-client grouping, gate groups):
    // one kernel per 8-bit pass, each tile's digit runs written contiguously
    // from LDS (the three-kernel sort's direct scatter: 173 us per pass over
    // config #3's 14.7M fanout pairs)
    if (tmp.os && hi_bit - lo_bit <= 32) return radix_sort2(k0, v0, k1, v1, n_max, n_dev, lo_bit, hi_bit, tmp.os, s);
    return radix_sort<uint32_t>(k0, v0, k1, v1, n_max, n_dev, lo_bit, hi_bit, tmp, s);
}

}  // namespace gw
