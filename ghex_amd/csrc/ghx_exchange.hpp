// ghx_exchange.hpp — the exchange plan behind the opaque ghx_exchange handle
// (communication_object::allocate semantics, include/ghex/communication_object.hpp:483-566,
// 1003-1067), shared by the C ABI (ghx_abi.cpp) and the per-peer pipeline (ghx_pipeline.cpp).
#pragma once

#include <memory>
#include <vector>

#include "ghx_plan.hpp"

namespace ghx
{
struct xbuffer
{
    int32_t first_id, second_id, rank, tag;
    uint64_t size = 0;
};

struct exchange_plan
{
    std::vector<xbuffer> send, recv;
    std::unique_ptr<splan> spack, sunpack;
    std::unique_ptr<uplan> upack, uunpack;
    // the fused self exchange's own pack/unpack plans when its tile size differs from the
    // two-launch path's (g_tune.self_tile_bytes); null = use spack/sunpack
    std::unique_ptr<splan> self_pack, self_unpack;
    // exchanges with self AND peer messages (build_mixed): per segment of spack the unpack
    // segment of its self message (zero = a peer message: pack only), and the unpack plan of
    // the peer messages alone
    device_tables mixed_comp;
    // pair records of the fused launches (upload_pair_records): the all-self exchange's
    // (ghx_exchange_self) and the mixed pack's (ghx_exchange_pack_self); empty: tile table path
    device_tables self_recs, mixed_recs;
    int mixed_max_field_slot = -1;  // the highest field slot mixed_comp's segments name
    std::unique_ptr<splan> punpack;
    bool mixed = false;
    parity_cfg mixed_parity;  // the mixed pack launch's double-buffered send buffers (direct)
    parity_cfg dir_parity[2];  // ghx_exchange_set_parity per direction (the per-buffer plans too)
    int32_t n_items = 0;
    mutable int self_ok = -1;  // lazily checked: may pack and unpack be fused (all self)?

    // The planner's entries per direction (0 send, 1 recv), kept for per-buffer plans; boxes
    // point into box_store, unstructured lids into the pattern (which outlives the exchange,
    // include/ghex/pattern_container.hpp:84-87).
    std::vector<ghx_pack_entry> entries[2];
    std::vector<std::vector<ghx_box>> box_store[2];
    std::vector<ghx_upack_entry> uentries[2];
    // per-buffer plans (ghx_exchange_split): [direction][buffer index], null = no bytes of
    // that kind in that buffer. The reference packs each buffer on its own stream
    // (include/ghex/communication_object.hpp:568-597, device/cuda/stream.hpp:25-73).
    std::vector<std::unique_ptr<splan>> bplan[2];
    std::vector<std::unique_ptr<uplan>> ubplan[2];
    bool split = false;

    void make_split()
    {
        if (split) return;
        for (int dir = 0; dir < 2; ++dir)
        {
            const size_t nb = dir == 0 ? send.size() : recv.size();
            bplan[dir].clear();
            ubplan[dir].clear();
            bplan[dir].resize(nb);
            ubplan[dir].resize(nb);
            for (size_t b = 0; b < nb; ++b)
            {
                std::vector<ghx_pack_entry> se;
                for (const auto& e : entries[dir])
                    if (size_t(e.buffer_slot) == b) se.push_back(e);
                std::vector<ghx_upack_entry> ue;
                for (const auto& e : uentries[dir])
                    if (size_t(e.buffer_slot) == b) ue.push_back(e);
                if (!se.empty()) bplan[dir][b] = std::make_unique<splan>(se.data(), int(se.size()), dir);
                if (!ue.empty()) ubplan[dir][b] = std::make_unique<uplan>(ue.data(), int(ue.size()), dir);
            }
        }
        split = true;
        for (int dir = 0; dir < 2; ++dir) set_split_parity(dir);
    }

    // the per-buffer plans use the copies ghx_exchange_set_parity selected, like the whole ones
    void set_split_parity(int dir)
    {
        for (auto& p : bplan[dir])
            if (p) p->parity = dir_parity[dir];
        for (auto& p : ubplan[dir])
            if (p) p->parity = dir_parity[dir];
    }

    // one buffer's pack (dir 0) or unpack (dir 1); the pointer arrays are the whole exchange's
    int execute_buffer(int dir, int b, void* const* fptr, int nf, void* const* bptr, int nb,
                       void* stream) const
    {
        if (!split) throw invalid("exchange is not split (ghx_exchange_split)");
        const size_t n = dir == 0 ? send.size() : recv.size();
        if (b < 0 || size_t(b) >= n) throw invalid("buffer index out of range");
        if (nb < int(n)) throw invalid("too few buffers");
        int rc = GHX_OK;
        if (bplan[dir][size_t(b)]) rc = bplan[dir][size_t(b)]->execute(fptr, nf, bptr, nb, stream);
        if (rc == GHX_OK && ubplan[dir][size_t(b)])
            rc = ubplan[dir][size_t(b)]->execute(fptr, nf, bptr, nb, stream);
        return rc;
    }

    // Every recv buffer aliases the send buffer of the same pair, and pack segment k and unpack
    // segment k cover the same buffer bytes (the launch tiles by the pack plan's table).
    bool self_fusable() const
    {
        if (self_ok >= 0) return self_ok == 1;
        bool ok = !upack && !uunpack && spack && sunpack && send.size() == recv.size() &&
                  !spack->grouped() && !sunpack->grouped();
        for (size_t i = 0; ok && i < send.size(); ++i)
            ok = send[i].first_id == recv[i].first_id && send[i].second_id == recv[i].second_id &&
                 send[i].size == recv[i].size;
        if (ok) ok = same_messages(*spack, *sunpack);
        self_ok = ok ? 1 : 0;
        return ok;
    }

    // Segment a of a launch's primary plan and its companion b (the unpack side of a fused self
    // tile, the target side of a put) cover the same buffer bytes with the same rows. Tiling is
    // deliberately not compared: a fused launch (k_self, k_put) runs the primary plan's tile
    // table and reads only a's tile_bytes, and the two sides size their short-row tiles from
    // different fields' row counts (a put's one source field vs one target field per peer; the
    // mixed pairing's self messages vs every message of the field), which differ once a field
    // holds more than the 512-row minimum's worth (512^3 (2,2,1) puts refused).
    static bool same_message(const seg_s& a, const seg_s& b)
    {
        return a.buf_slot == b.buf_slot && a.buf_off == b.buf_off && a.bytes == b.bytes &&
               a.row_bytes == b.row_bytes;
    }

    // pack segment k and unpack segment k cover the same buffer bytes (same_message)
    static bool same_messages(const splan& p, const splan& q)
    {
        bool ok = p.host_segs.size() == q.host_segs.size();
        for (size_t k = 0; ok && k < p.host_segs.size(); ++k)
            ok = same_message(p.host_segs[k], q.host_segs[k]);
        return ok;
    }
};
}  // namespace ghx

struct ghx_exchange : ghx::exchange_plan
{
};
