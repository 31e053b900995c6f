// ghx_abi.cpp — the extern "C" boundary (include/ghx.h): argument checks, error capture,
// opaque handles, and the exchange planner (communication_object::allocate semantics).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <list>
#include <map>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <unordered_map>
#include <vector>

#include "ghx_exchange.hpp"
#include "ghx_guard.hpp"
#include "ghx_pattern.hpp"
#include "ghx_plan.hpp"

namespace ghx
{
namespace
{
// Plan caches of the per-call convenience entry points (ghx_structured_pack/unpack,
// ghx_unstructured_pack/unpack), like the reference's pattern container that outlives its
// exchanges (include/ghex/pattern_container.hpp:84-87). A hit is exact: the structured key IS
// the content (descriptor, iteration spaces, direction); the unstructured entry keeps a host
// copy of its index list and compares it in full on every hit, so a list mutated in place gets
// a fresh plan. Evicted or replaced plans are never freed under the lock with a device-wide
// synchronisation: they are retired and freed once every stream that executed them has passed
// the event recorded after its last execution there (plans executed inside a stream capture are
// kept: a graph may still reference their device tables).
template<typename Plan>
struct cached_plan
{
    struct use
    {
        hipStream_t stream;
        hipEvent_t done;  // recorded after the latest execution on `stream`
    };
    std::unique_ptr<Plan> plan;
    std::vector<char> content;  // unstructured: the index list bytes the plan was built from
    std::vector<use> uses;      // one record per stream that has executed the plan
    bool captured = false;
    bool idle() const
    {
        for (const auto& u : uses)
            if (hipEventQuery(u.done) != hipSuccess) return false;
        return true;
    }
    ~cached_plan()
    {
        for (auto& u : uses) (void)hipEventDestroy(u.done);
    }
};

template<typename Plan>
class plan_lru
{
    using entry = std::shared_ptr<cached_plan<Plan>>;
    std::mutex mtx_;
    std::list<std::string> lru_;
    std::unordered_map<std::string, std::pair<entry, std::list<std::string>::iterator>> map_;
    std::vector<entry> retired_;
    static constexpr size_t kCap = 256;

    void retire(entry e) { retired_.push_back(std::move(e)); }
    void reap()  // free retired plans nobody holds whose last execution has completed
    {
        std::vector<entry> keep;
        for (auto& e : retired_)
        {
            const bool idle = e.use_count() == 1 && !e->captured && e->idle();
            if (!idle) keep.push_back(std::move(e));
        }
        retired_.swap(keep);
    }

  public:
    // the cached entry for `key` if `same(entry)` holds, else the one `make()` builds
    template<typename Same, typename Make>
    entry get(const std::string& key, Same&& same, Make&& make)
    {
        {
            std::lock_guard<std::mutex> lk(mtx_);
            auto it = map_.find(key);
            if (it != map_.end() && same(*it->second.first))
            {
                lru_.splice(lru_.begin(), lru_, it->second.second);
                return it->second.first;
            }
        }
        entry fresh = make();  // plan construction (device upload) outside the lock
        std::lock_guard<std::mutex> lk(mtx_);
        reap();
        auto it = map_.find(key);
        if (it != map_.end())
        {
            retire(it->second.first);  // stale content (or built concurrently): replace
            lru_.erase(it->second.second);
            map_.erase(it);
        }
        if (map_.size() >= kCap)
        {
            auto old = map_.find(lru_.back());
            retire(old->second.first);
            map_.erase(old);
            lru_.pop_back();
        }
        lru_.push_front(key);
        map_.emplace(key, std::make_pair(fresh, lru_.begin()));
        return fresh;
    }

    // stream-ordered record of a use (no host synchronisation). One event per stream: a later
    // execution on the same stream is ordered after the earlier ones, so re-recording that
    // stream's event keeps covering them; an execution on another stream gets its own record,
    // so a plan used on streams A then B is freed only once BOTH have passed their last use.
    void used(cached_plan<Plan>& c, void* stream)
    {
        hipStream_t s = static_cast<hipStream_t>(stream);
        hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
        (void)hipStreamIsCapturing(s, &st);
        std::lock_guard<std::mutex> lk(mtx_);
        if (st != hipStreamCaptureStatusNone)
        {
            c.captured = true;
            return;
        }
        for (auto& u : c.uses)
            if (u.stream == s)
            {
                if (hipEventRecord(u.done, s) != hipSuccess) c.captured = true;
                return;
            }
        // a new stream: drop the records of streams that have passed their last use (bounds
        // the list for callers that rotate through many streams)
        std::vector<typename cached_plan<Plan>::use> live;
        for (auto& u : c.uses)
        {
            if (hipEventQuery(u.done) == hipSuccess) (void)hipEventDestroy(u.done);
            else live.push_back(u);
        }
        c.uses.swap(live);
        hipEvent_t e = nullptr;
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess)
        {
            c.captured = true;  // cannot track it: never free it
            return;
        }
        if (hipEventRecord(e, s) != hipSuccess)
        {
            (void)hipEventDestroy(e);
            c.captured = true;
            return;
        }
        c.uses.push_back({s, e});
    }
};

plan_lru<splan>& cache()
{
    static plan_lru<splan> c;
    return c;
}

plan_lru<uplan>& ucache()
{
    static plan_lru<uplan> c;
    return c;
}

int run_structured(const ghx_field_desc& f, const ghx_box* boxes, int n, int dir, void* field,
                   void* buffer, void* stream)
{
    std::string key(reinterpret_cast<const char*>(&f), sizeof(f));
    key.append(reinterpret_cast<const char*>(boxes), sizeof(ghx_box) * size_t(n));
    key.push_back(char(dir));
    auto c = cache().get(
        key, [](const cached_plan<splan>&) { return true; },
        [&] {
            ghx_pack_entry e{};
            e.field = f;
            e.boxes = boxes;
            e.n_boxes = n;
            auto p = std::make_shared<cached_plan<splan>>();
            p->plan = std::make_unique<splan>(&e, 1, dir);
            return p;
        });
    void* fp[1] = {field};
    void* bp[1] = {buffer};
    const int rc = c->plan->execute(fp, 1, bp, 1, stream);
    cache().used(*c, stream);
    return rc;
}

int run_unstructured(const ghx_udata_desc& d, const void* lids, int32_t lid_bytes, int64_t n,
                     int dir, void* values, void* buffer, void* stream)
{
    std::string key(reinterpret_cast<const char*>(&d), sizeof(d));
    const uint64_t meta[4] = {uint64_t(reinterpret_cast<uintptr_t>(lids)), uint64_t(n),
                              uint64_t(lid_bytes), uint64_t(dir)};
    key.append(reinterpret_cast<const char*>(meta), sizeof(meta));
    const size_t nbytes = size_t(n) * size_t(lid_bytes);
    auto c = ucache().get(
        key,
        [&](const cached_plan<uplan>& e) {
            return e.content.size() == nbytes && std::memcmp(e.content.data(), lids, nbytes) == 0;
        },
        [&] {
            std::vector<int64_t> wide;
            const int64_t* l64 = static_cast<const int64_t*>(lids);
            if (lid_bytes == 4)
            {
                wide.resize(size_t(n));
                for (int64_t i = 0; i < n; ++i) wide[size_t(i)] = static_cast<const int32_t*>(lids)[i];
                l64 = wide.data();
            }
            ghx_upack_entry e{};
            e.data = d;
            e.lids = l64;
            e.n_lids = n;
            auto p = std::make_shared<cached_plan<uplan>>();
            p->plan = std::make_unique<uplan>(&e, 1, dir);
            p->content.assign(static_cast<const char*>(lids), static_cast<const char*>(lids) + nbytes);
            return p;
        });
    void* fp[1] = {values};
    void* bp[1] = {buffer};
    const int rc = c->plan->execute(fp, 1, bp, 1, stream);
    ucache().used(*c, stream);
    return rc;
}
}  // namespace

namespace
{
thread_local std::string g_error;
}
void set_error(const std::string& msg) { g_error = msg; }
const char* get_error() { return g_error.c_str(); }

}  // namespace ghx

// Put plan: the pack plan of the source side and the unpack plan of the target side, segment k
// of each covering the same virtual message bytes (checked). The launch is tiled by the source
// plan's tile table alone (k_put addresses the target segment by message position), so the
// target plan's own tiling is not compared: the two sides size their short-row tiles by their
// own fields' rows (one source field, one target field per peer) and differ at large sizes.
struct ghx_put
{
    std::unique_ptr<ghx::splan> from, to;
    ghx_put(const ghx_pack_entry* src, int n_src, const ghx_pack_entry* dst, int n_dst)
    : from(new ghx::splan(src, n_src, 0)), to(new ghx::splan(dst, n_dst, 1))
    {
        bool ok = from->host_segs.size() == to->host_segs.size() && from->bytes == to->bytes;
        for (size_t k = 0; ok && k < from->host_segs.size(); ++k)
        {
            const auto& a = from->host_segs[k];
            const auto& b = to->host_segs[k];
            ok = ghx::exchange_plan::same_message(a, b) && a.n_outer == b.n_outer;
            for (int d = 0; ok && d < 4; ++d) ok = a.ext[d] == b.ext[d];
        }
        if (!ok)
            throw ghx::invalid("source and target iteration spaces do not describe the same "
                               "message bytes (shapes, order, element sizes or row structure differ)");
        if (from->grouped() || to->grouped())
            throw ghx::invalid("a put plan takes at most 64 source and 64 target fields (one launch)");
        ghx::upload_pair_records(recs, from->host_segs, to->host_segs, from->host_tiles);
    }
    ghx::device_tables recs;  // pair records (source segment with tile index, target segment)
};

using namespace ghx;

namespace
{
// communication_object::allocate (include/ghex/communication_object.hpp:1019-1066)
void plan_direction(const ghx_exchange_item* items, int n_items, bool receive,
                    std::vector<xbuffer>& bufs_out, std::vector<ghx_pack_entry>& sent,
                    std::vector<ghx_upack_entry>& uent, std::vector<std::vector<ghx_box>>& box_store)
{
    struct finfo
    {
        int item;
        const halo_entry* e;
        uint64_t offset;
    };
    struct buf
    {
        xbuffer x;
        std::vector<finfo> fields;
    };
    std::map<std::pair<int32_t, int32_t>, buf> mem;  // domain_id_pair ordering (:165-174)
    for (int k = 0; k < n_items; ++k)
    {
        const auto& it = items[k];
        if (!it.pattern) throw invalid("exchange item without pattern");
        const auto& ps = *it.pattern;
        if (it.local_index < 0 || it.local_index >= int(ps.doms.size()))
            throw invalid("exchange item local_index out of range");
        if ((it.kind == 0) != (ps.kind == 0)) throw invalid("field kind does not match pattern kind");
        if (it.align < 1 || (it.align & (it.align - 1))) throw invalid("align must be a power of two");
        const auto& dp = ps.doms[size_t(it.local_index)];
        const auto& halos = receive ? dp.recv : dp.send;
        int64_t nc, elem;
        if (it.kind == 0)
        {
            validate_field(it.field);
            nc = it.field.num_components;
            elem = it.field.elem_size;
        }
        else
        {
            nc = it.udata.levels;
            elem = it.udata.elem_size;
        }
        for (const auto& e : halos)
        {
            int64_t n = 0;
            if (it.kind == 0)
                for (const auto& b : e.boxes) n += b.size(ps.dim);
            else n = int64_t(e.lids.size());
            n *= nc;
            if (n < 1) continue;
            const auto pair = receive ? std::make_pair(dp.id, e.key.remote_id)
                                      : std::make_pair(e.key.remote_id, dp.id);
            auto bi = mem.find(pair);
            if (bi == mem.end())
            {
                buf b;
                b.x = {pair.first, pair.second, e.key.remote_rank, e.key.tag + it.tag_offset, 0};
                bi = mem.emplace(pair, std::move(b)).first;
            }
            const uint64_t prev = bi->second.x.size;
            const uint64_t a = uint64_t(it.align);
            const uint64_t pad = ((prev + a - 1) / a) * a - prev;
            bi->second.fields.push_back({k, &e, prev + pad});
            bi->second.x.size += pad + uint64_t(n) * uint64_t(elem);
        }
    }
    int32_t slot = 0;
    for (auto& kv : mem)
    {
        bufs_out.push_back(kv.second.x);
        for (const auto& fi : kv.second.fields)
        {
            const auto& it = items[fi.item];
            if (it.kind == 0)
            {
                const int dim = it.pattern->dim;
                box_store.emplace_back();
                auto& bx = box_store.back();
                for (const auto& b : fi.e->boxes)
                {
                    ghx_box g{};
                    for (int d = 0; d < dim; ++d)
                    {
                        g.first[d] = b.lf[d];
                        g.last[d] = b.ll[d];
                    }
                    bx.push_back(g);
                }
                if (it.field.dim - (it.field.has_components ? 1 : 0) != dim)
                    throw invalid("field spatial dimension does not match the pattern");
                ghx_pack_entry pe{};
                pe.field = it.field;
                pe.field_slot = fi.item;
                pe.buffer_slot = slot;
                pe.buffer_offset = fi.offset;
                pe.boxes = bx.data();
                pe.n_boxes = int32_t(bx.size());
                sent.push_back(pe);
            }
            else
            {
                ghx_upack_entry ue{};
                ue.data = it.udata;
                ue.field_slot = fi.item;
                ue.buffer_slot = slot;
                ue.buffer_offset = fi.offset;
                ue.lids = fi.e->lids.data();
                ue.n_lids = int64_t(fi.e->lids.size());
                uent.push_back(ue);
            }
        }
        ++slot;
    }
}

// Exchanges with self AND peer messages — a rank whose periodic wrap reaches itself next to real
// neighbours, e.g. the (2,1,1) and (2,2,1) decompositions: the pack launch also writes the halos
// of the self messages straight from the registers it packs them from (k_self's forwarding path),
// and the unpack launch covers the peer messages only. Companion segment k of the pack plan is
// the unpack segment of the same buffer bytes for a self message (same tiling, checked), or
// zero for a peer message. `rent` = the receive-side pack entries of every recv buffer.
void build_mixed(exchange_plan& ex, int32_t me, const std::vector<ghx_pack_entry>& rent)
{
    if (!ex.spack || !ex.sunpack || ex.upack || ex.uunpack || me < 0 || ex.self_fusable()) return;
    std::vector<int> send_of_recv(ex.recv.size(), -1);
    bool any_self = false;
    for (size_t j = 0; j < ex.recv.size(); ++j)
    {
        const xbuffer& r = ex.recv[j];
        if (r.rank != me) continue;
        for (size_t i = 0; i < ex.send.size(); ++i)
        {
            const xbuffer& s = ex.send[i];
            if (s.rank == me && s.first_id == r.first_id && s.second_id == r.second_id &&
                s.size == r.size)
            {
                send_of_recv[j] = int(i);
                any_self = true;
                break;
            }
        }
    }
    if (!any_self) return;
    std::vector<ghx_pack_entry> self_e, peer_e;
    for (const ghx_pack_entry& e : rent)
    {
        const int i = send_of_recv[size_t(e.buffer_slot)];
        if (i < 0)
        {
            peer_e.push_back(e);
            continue;
        }
        ghx_pack_entry s = e;
        s.buffer_slot = i;  // a self message's recv buffer IS its send buffer
        self_e.push_back(s);
    }
    if (peer_e.empty()) return;
    std::stable_sort(self_e.begin(), self_e.end(),
                     [](const ghx_pack_entry& a, const ghx_pack_entry& b) {
                         return a.buffer_slot < b.buffer_slot;
                     });
    if (ex.spack->grouped()) return;  // more slots than one launch holds: two-launch path
    const splan su(self_e.data(), int(self_e.size()), 1);
    if (su.grouped()) return;
    std::vector<char> is_self(ex.send.size(), 0);
    for (int i : send_of_recv)
        if (i >= 0) is_self[size_t(i)] = 1;
    const std::vector<seg_s>& ps = ex.spack->host_segs;
    std::vector<seg_s> comp(ps.size());  // value-initialised: bytes = 0 -> pack only
    size_t m = 0;
    bool short_self = false;
    for (size_t k = 0; k < ps.size(); ++k)
    {
        if (!is_self[ps[k].buf_slot]) continue;
        short_self = short_self || ps[k].row_bytes < g_tune.small_row_bytes;
        if (m >= su.host_segs.size()) return;
        const seg_s& q = su.host_segs[m++];
        if (!exchange_plan::same_message(ps[k], q) || q.bytes == 0) return;
        comp[k] = q;
    }
    if (m != su.host_segs.size()) return;
    // Worth it only when the self messages include request-bound short rows (the unit-stride
    // x-faces of an x-local decomposition such as (1,1,2)): fusing their reads and writes into
    // one launch is what the fused self exchange gains. Self messages of long rows alone (the
    // y/z wrap of a (2,1,1) decomposition) measured 1-3 % slower mixed than plain
    // (tools/emu_rank_bench.py, profiles/r01c_emu_rank.jsonl).
    if (!short_self && !g_tune.mixed_always) return;
    upload_segments(ex.mixed_comp, comp);
    upload_pair_records(ex.mixed_recs, ps, comp, ex.spack->host_tiles);
    ex.mixed_max_field_slot = su.max_field_slot;
    ex.punpack = std::make_unique<splan>(peer_e.data(), int(peer_e.size()), 1);
    ex.mixed = true;
}

int check_ptr(const void* p, const char* what)
{
    if (!p) throw invalid(std::string("null argument: ") + what);
    return 0;
}
}  // namespace

extern "C" {

const char* ghx_last_error(void) { return ghx::get_error(); }

const char* ghx_version(void) { return "ghex_amd 0.1.0 (gfx950)"; }

int ghx_tune(const char* key, int32_t value)
{
    return guarded([&] {
        check_ptr(key, "key");
        const std::string k(key);
        if (k == "reset")
            g_tune = tuning{};
        else if (k == "order")
        {
            if (value < 0 || value > 1) throw invalid("order must be 0 or 1");
            g_tune.order = value;
        }
        else if (k == "self_tile_bytes")
        {
            if (value < 1024 || uint32_t(value) > kMaxTileBytes || (value & (value - 1)))
                throw invalid("self_tile_bytes must be a power of two in [1 KiB, 1 MiB]");
            g_tune.self_tile_bytes = uint32_t(value);
        }
        else if (k == "mixed_always")
        {
            if (value < 0 || value > 1) throw invalid("mixed_always must be 0 or 1");
            g_tune.mixed_always = value;
        }
        else if (k == "unpack_tile_bytes")
        {
            if (value != 0 && (value < 1024 || uint32_t(value) > kMaxTileBytes || (value & (value - 1))))
                throw invalid("unpack_tile_bytes must be 0 or a power of two in [1 KiB, 1 MiB]");
            g_tune.unpack_tile_bytes = uint32_t(value);
        }
        else if (k == "tile_records")
        {
            if (value < 0 || value > 1) throw invalid("tile_records must be 0 or 1");
            g_tune.tile_records = value;
        }
        else if (k == "pack_tile_rows")
        {
            if (value != 0 && (value < 64 || value > 65536))
                throw invalid("pack_tile_rows must be 0 (as small_tile_rows) or in [64, 65536]");
            g_tune.pack_tile_rows = uint32_t(value);
        }
        else if (k == "unpack_tile_rows")
        {
            if (value != 0 && (value < 64 || value > 65536))
                throw invalid("unpack_tile_rows must be 0 (as small_tile_rows) or in [64, 65536]");
            g_tune.unpack_tile_rows = uint32_t(value);
        }
        else if (k == "fast_addr")
        {
            if (value < 0 || value > 1) throw invalid("fast_addr must be 0 or 1");
            g_tune.fast_addr = value;
        }
        else if (k == "xcd_pair")
        {
            if (value < 0 || value > 1) throw invalid("xcd_pair must be 0 or 1");
            g_tune.xcd_pair = value;
        }
        else if (k == "u_tile_rows")
        {
            if (value < 1) throw invalid("u_tile_rows must be >= 1");
            g_tune.u_tile_rows = uint32_t(value);
        }
        else if (k == "u_tile_bytes")
        {
            if (value < 1024 || uint32_t(value) > kMaxTileBytes || (value & (value - 1)))
                throw invalid("u_tile_bytes must be a power of two in [1 KiB, 1 MiB]");
            g_tune.u_tile_bytes = uint32_t(value);
        }
        else if (k == "urun")
        {
            if (value < 0 || value > 1) throw invalid("urun must be 0 or 1");
            g_tune.urun = value;
        }
        else if (k == "u_run_tile_rows")
        {
            if (value < 4) throw invalid("u_run_tile_rows must be >= 4");
            g_tune.u_run_tile_rows = uint32_t(value);
        }
        else if (k == "short_pol")
        {
            if (value < 0 || value > 3) throw invalid("short_pol must be in 0..3");
            g_tune.short_pol = value;
        }
        else if (k == "small_row_bytes")
        {
            if (value < 1) throw invalid("small_row_bytes must be >= 1");
            g_tune.small_row_bytes = uint32_t(value);
        }
        else if (k == "small_tile_rows")
        {
            if (value != 0 && (value < 64 || value > (1 << 16)))
                throw invalid("small_tile_rows must be 0 (auto) or in [64, 65536]");
            g_tune.small_tile_rows = uint32_t(value);
        }
        else if (k == "grid_cap")
        {
            if (value < 0) throw invalid("grid_cap must be >= 0");
            g_tune.grid_cap = value;
        }
        else if (k == "tile_bytes")
        {
            if (value < 1024 || uint32_t(value) > kMaxTileBytes || (value & (value - 1)))
                throw invalid("tile_bytes must be a power of two in [1 KiB, 1 MiB]");
            g_tune.tile_bytes = uint32_t(value);
        }
        else throw invalid("unknown tuning key: " + k);
        return GHX_OK;
    });
}

int ghx_launch_timing(int32_t enable)
{
    return guarded([&] {
        ghx::timing_enable(enable != 0);
        return GHX_OK;
    });
}

int ghx_launch_timing_read(float* ms, int32_t cap, int32_t* n)
{
    return guarded([&] {
        if (cap < 0 || (cap > 0 && !ms)) throw invalid("bad ms / cap");
        return ghx::timing_read(ms, cap, n);
    });
}

int ghx_plan_create(const ghx_pack_entry* entries, int32_t n_entries, int32_t direction,
                    ghx_plan** out)
{
    return guarded([&] {
        check_ptr(out, "out");
        if (n_entries < 0 || (n_entries > 0 && !entries)) throw invalid("bad entries");
        *out = new ghx_plan(entries, n_entries, direction);
        return GHX_OK;
    });
}

int ghx_plan_execute(const ghx_plan* plan, void* const* field_ptrs, int32_t n_field_ptrs,
                     void* const* buffer_ptrs, int32_t n_buffer_ptrs, ghx_stream stream)
{
    return guarded([&] {
        check_ptr(plan, "plan");
        return plan->execute(field_ptrs, n_field_ptrs, buffer_ptrs, n_buffer_ptrs, stream);
    });
}

int ghx_plan_destroy(ghx_plan* plan)
{
    return guarded([&] {
        delete plan;
        return GHX_OK;
    });
}

int ghx_plan_info(const ghx_plan* plan, uint64_t* bytes, int32_t* n_segments, int32_t* n_tiles)
{
    return guarded([&] {
        check_ptr(plan, "plan");
        if (bytes) *bytes = plan->bytes;
        if (n_segments) *n_segments = plan->n_segments;
        if (n_tiles) *n_tiles = int32_t(plan->total_tiles());
        return GHX_OK;
    });
}

int ghx_structured_pack(const ghx_field_desc* field, const void* field_data, void* buffer,
                        const ghx_box* boxes, int32_t n_boxes, ghx_stream stream)
{
    return guarded([&] {
        check_ptr(field, "field");
        if (n_boxes < 0 || (n_boxes > 0 && !boxes)) throw invalid("bad boxes");
        return run_structured(*field, boxes, n_boxes, 0, const_cast<void*>(field_data), buffer,
                              stream);
    });
}

int ghx_structured_unpack(const ghx_field_desc* field, void* field_data, const void* buffer,
                          const ghx_box* boxes, int32_t n_boxes, ghx_stream stream)
{
    return guarded([&] {
        check_ptr(field, "field");
        if (n_boxes < 0 || (n_boxes > 0 && !boxes)) throw invalid("bad boxes");
        return run_structured(*field, boxes, n_boxes, 1, field_data, const_cast<void*>(buffer),
                              stream);
    });
}

int ghx_unstructured_pack(const ghx_udata_desc* data, const void* values, void* buffer,
                          const void* lids, int32_t lid_bytes, int64_t n_lids, ghx_stream stream)
{
    return guarded([&] {
        check_ptr(data, "data");
        if (lid_bytes != 4 && lid_bytes != 8) throw invalid("lid_bytes must be 4 or 8");
        if (n_lids < 0 || (n_lids > 0 && !lids)) throw invalid("bad index list");
        if (n_lids == 0) return int(GHX_OK);
        return run_unstructured(*data, lids, lid_bytes, n_lids, 0, const_cast<void*>(values),
                                buffer, stream);
    });
}

int ghx_unstructured_unpack(const ghx_udata_desc* data, void* values, const void* buffer,
                            const void* lids, int32_t lid_bytes, int64_t n_lids, ghx_stream stream)
{
    return guarded([&] {
        check_ptr(data, "data");
        if (lid_bytes != 4 && lid_bytes != 8) throw invalid("lid_bytes must be 4 or 8");
        if (n_lids < 0 || (n_lids > 0 && !lids)) throw invalid("bad index list");
        if (n_lids == 0) return int(GHX_OK);
        return run_unstructured(*data, lids, lid_bytes, n_lids, 1, values,
                                const_cast<void*>(buffer), stream);
    });
}

int ghx_uplan_create(const ghx_upack_entry* entries, int32_t n_entries, int32_t direction,
                     ghx_uplan** out)
{
    return guarded([&] {
        check_ptr(out, "out");
        if (n_entries < 0 || (n_entries > 0 && !entries)) throw invalid("bad entries");
        *out = new ghx_uplan(entries, n_entries, direction);
        return GHX_OK;
    });
}

int ghx_uplan_execute(const ghx_uplan* plan, void* const* field_ptrs, int32_t n_field_ptrs,
                      void* const* buffer_ptrs, int32_t n_buffer_ptrs, ghx_stream stream)
{
    return guarded([&] {
        check_ptr(plan, "plan");
        return plan->execute(field_ptrs, n_field_ptrs, buffer_ptrs, n_buffer_ptrs, stream);
    });
}

int ghx_uplan_destroy(ghx_uplan* plan)
{
    return guarded([&] {
        delete plan;
        return GHX_OK;
    });
}

int ghx_uplan_info(const ghx_uplan* plan, uint64_t* bytes, int32_t* n_segments, int32_t* n_tiles)
{
    return guarded([&] {
        check_ptr(plan, "plan");
        if (bytes) *bytes = plan->bytes;
        if (n_segments) *n_segments = plan->n_segments;
        if (n_tiles) *n_tiles = int32_t(plan->total_tiles());
        return GHX_OK;
    });
}

// ----------------------------------------------------------------------------------- patterns
int ghx_regular_halo_boxes(int32_t dim, const int32_t* global_first, const int32_t* global_last,
                           const int32_t* halos, const int32_t* periodic,
                           const int32_t* domain_first, const int32_t* domain_last,
                           ghx_box* local, ghx_box* global, int32_t max_boxes, int32_t* n_boxes)
{
    return guarded([&] {
        if (dim < 1 || dim > 3) throw invalid("dim must be 1, 2 or 3");
        check_ptr(global_first, "global_first");
        check_ptr(global_last, "global_last");
        check_ptr(halos, "halos");
        check_ptr(periodic, "periodic");
        check_ptr(domain_first, "domain_first");
        check_ptr(domain_last, "domain_last");
        check_ptr(n_boxes, "n_boxes");
        auto b = regular_halo_boxes(dim, global_first, global_last, halos, periodic, domain_first,
                                    domain_last);
        *n_boxes = int32_t(b.size());
        for (int32_t i = 0; i < std::min<int32_t>(max_boxes, int32_t(b.size())); ++i)
        {
            ghx_box l{}, g{};
            for (int d = 0; d < dim; ++d)
            {
                l.first[d] = b[i].lf[d];
                l.last[d] = b[i].ll[d];
                g.first[d] = b[i].gf[d];
                g.last[d] = b[i].gl[d];
            }
            if (local) local[i] = l;
            if (global) global[i] = g;
        }
        return GHX_OK;
    });
}

int ghx_regular_pattern_create(int32_t dim, const ghx_regular_domain* domains,
                               int32_t n_domains, const int32_t* global_first,
                               const int32_t* global_last, const int32_t* halos,
                               const int32_t* periodic, int32_t my_rank, ghx_pattern** out)
{
    return guarded([&] {
        check_ptr(out, "out");
        check_ptr(domains, "domains");
        check_ptr(global_first, "global_first");
        check_ptr(global_last, "global_last");
        check_ptr(halos, "halos");
        check_ptr(periodic, "periodic");
        if (dim < 1 || dim > 3) throw invalid("dim must be 1, 2 or 3");
        if (n_domains < 1) throw invalid("need at least one domain");
        for (int i = 0; i < n_domains; ++i)
            for (int j = 0; j < i; ++j)
                if (domains[i].id == domains[j].id) throw invalid("domain ids must be unique");
        auto p = std::make_unique<ghx_pattern>();
        regular_make_pattern(dim, domains, n_domains, global_first, global_last, halos, periodic,
                             my_rank, *p);
        *out = p.release();
        return GHX_OK;
    });
}

int ghx_staged_pattern_create(int32_t dim, const ghx_regular_domain* domains, int32_t n_domains,
                              const int32_t* neighbors, const int32_t* global_first,
                              const int32_t* global_last, const int32_t* halos,
                              const int32_t* periodic, int32_t my_rank, ghx_pattern** out)
{
    return guarded([&] {
        check_ptr(out, "out");
        check_ptr(domains, "domains");
        check_ptr(neighbors, "neighbors");
        check_ptr(global_first, "global_first");
        check_ptr(global_last, "global_last");
        check_ptr(halos, "halos");
        check_ptr(periodic, "periodic");
        if (dim < 1 || dim > 3) throw invalid("dim must be 1, 2 or 3");
        if (n_domains < 1) throw invalid("need at least one domain");
        std::vector<ghx::pattern_set> sets;
        try
        {
            ghx::staged_make_pattern(dim, domains, n_domains, neighbors, global_first,
                                     global_last, halos, periodic, my_rank, sets);
        }
        catch (const std::runtime_error& e)
        {
            throw invalid(e.what());
        }
        std::vector<std::unique_ptr<ghx_pattern>> ps;
        for (auto& s : sets)
        {
            ps.push_back(std::make_unique<ghx_pattern>());
            static_cast<ghx::pattern_set&>(*ps.back()) = std::move(s);
        }
        for (int i = 0; i < dim; ++i) out[i] = ps[i].release();
        return GHX_OK;
    });
}

int ghx_pattern_filter(const ghx_pattern* p, const int32_t* ranks, int32_t n_ranks, int32_t keep,
                       ghx_pattern** out)
{
    return guarded([&] {
        check_ptr(p, "pattern");
        check_ptr(out, "out");
        if (n_ranks < 0 || (n_ranks > 0 && !ranks)) throw invalid("bad rank list");
        if (keep != 0 && keep != 1) throw invalid("keep must be 0 or 1");
        auto in_set = [&](int32_t r) {
            for (int32_t i = 0; i < n_ranks; ++i)
                if (ranks[i] == r) return true;
            return false;
        };
        auto q = std::make_unique<ghx_pattern>();
        static_cast<pattern_set&>(*q) = static_cast<const pattern_set&>(*p);
        for (auto& d : q->doms)
            for (auto* v : {&d.send, &d.recv})
            {
                std::vector<halo_entry> kept;
                for (auto& e : *v)
                    if (in_set(e.key.remote_rank) == (keep == 1)) kept.push_back(std::move(e));
                v->swap(kept);
            }
        *out = q.release();
        return GHX_OK;
    });
}

int ghx_pattern_destroy(ghx_pattern* p)
{
    return guarded([&] {
        delete p;
        return GHX_OK;
    });
}

int ghx_pattern_num_domains(const ghx_pattern* p, int32_t* n)
{
    return guarded([&] {
        check_ptr(p, "pattern");
        check_ptr(n, "n");
        *n = int32_t(p->doms.size());
        return GHX_OK;
    });
}

int ghx_pattern_max_tag(const ghx_pattern* p, int32_t* max_tag)
{
    return guarded([&] {
        check_ptr(p, "pattern");
        check_ptr(max_tag, "max_tag");
        *max_tag = p->max_tag;
        return GHX_OK;
    });
}

int ghx_pattern_domain_id(const ghx_pattern* p, int32_t local_index, int32_t* id)
{
    return guarded([&] {
        check_ptr(p, "pattern");
        check_ptr(id, "id");
        if (local_index < 0 || local_index >= int32_t(p->doms.size())) throw invalid("local_index");
        *id = p->doms[size_t(local_index)].id;
        return GHX_OK;
    });
}

static const ghx::halo_entry& key_of(const ghx_pattern* p, int32_t li, int32_t dir, int32_t key)
{
    if (!p) throw invalid("null pattern");
    if (li < 0 || li >= int32_t(p->doms.size())) throw invalid("local_index out of range");
    const auto& v = dir == 0 ? p->doms[size_t(li)].send : p->doms[size_t(li)].recv;
    if (key < 0 || key >= int32_t(v.size())) throw invalid("key out of range");
    return v[size_t(key)];
}

int ghx_pattern_num_keys(const ghx_pattern* p, int32_t local_index, int32_t direction,
                         int32_t* n_keys)
{
    return guarded([&] {
        check_ptr(p, "pattern");
        check_ptr(n_keys, "n_keys");
        if (local_index < 0 || local_index >= int32_t(p->doms.size())) throw invalid("local_index");
        const auto& d = p->doms[size_t(local_index)];
        *n_keys = int32_t(direction == 0 ? d.send.size() : d.recv.size());
        return GHX_OK;
    });
}

int ghx_pattern_key(const ghx_pattern* p, int32_t local_index, int32_t direction, int32_t key,
                    int32_t* remote_id, int32_t* remote_rank, int32_t* tag, int32_t* n_spaces,
                    int64_t* n_elements)
{
    return guarded([&] {
        const auto& e = key_of(p, local_index, direction, key);
        if (remote_id) *remote_id = e.key.remote_id;
        if (remote_rank) *remote_rank = e.key.remote_rank;
        if (tag) *tag = e.key.tag;
        if (p->kind == 0)
        {
            if (n_spaces) *n_spaces = int32_t(e.boxes.size());
            if (n_elements)
            {
                int64_t n = 0;
                for (const auto& b : e.boxes) n += b.size(p->dim);
                *n_elements = n;
            }
        }
        else
        {
            if (n_spaces) *n_spaces = 1;
            if (n_elements) *n_elements = int64_t(e.lids.size());
        }
        return GHX_OK;
    });
}

int ghx_pattern_key_boxes(const ghx_pattern* p, int32_t local_index, int32_t direction,
                          int32_t key, ghx_box* local, ghx_box* global, int32_t max_boxes)
{
    return guarded([&] {
        const auto& e = key_of(p, local_index, direction, key);
        if (p->kind != 0) throw invalid("not a structured pattern");
        for (int32_t i = 0; i < std::min<int32_t>(max_boxes, int32_t(e.boxes.size())); ++i)
        {
            ghx_box l{}, g{};
            for (int d = 0; d < p->dim; ++d)
            {
                l.first[d] = e.boxes[size_t(i)].lf[d];
                l.last[d] = e.boxes[size_t(i)].ll[d];
                g.first[d] = e.boxes[size_t(i)].gf[d];
                g.last[d] = e.boxes[size_t(i)].gl[d];
            }
            if (local) local[i] = l;
            if (global) global[i] = g;
        }
        return GHX_OK;
    });
}

int ghx_pattern_key_lids(const ghx_pattern* p, int32_t local_index, int32_t direction,
                         int32_t key, int64_t* lids, int64_t max_lids)
{
    return guarded([&] {
        const auto& e = key_of(p, local_index, direction, key);
        if (p->kind != 1) throw invalid("not an unstructured pattern");
        check_ptr(lids, "lids");
        const int64_t n = std::min<int64_t>(max_lids, int64_t(e.lids.size()));
        std::memcpy(lids, e.lids.data(), size_t(n) * sizeof(int64_t));
        return GHX_OK;
    });
}

// ---------------------------------------------------------------------------------- exchange
int ghx_exchange_create(const ghx_exchange_item* items, int32_t n_items, ghx_exchange** out)
{
    return guarded([&] {
        check_ptr(out, "out");
        if (n_items < 1 || !items) throw invalid("need at least one exchange item");
        auto ex = std::make_unique<ghx_exchange>();
        ex->n_items = n_items;
        std::vector<ghx_pack_entry> rent;              // receive entries, for build_mixed
        for (int dir = 0; dir < 2; ++dir)
        {
            const bool receive = dir == 1;
            std::vector<ghx_pack_entry> sent;
            std::vector<ghx_upack_entry> uent;
            std::vector<std::vector<ghx_box>> store;
            store.reserve(size_t(n_items) * 64);
            auto& bufs = receive ? ex->recv : ex->send;
            plan_direction(items, n_items, receive, bufs, sent, uent, store);
            // kept for per-buffer plans (ghx_exchange_split); moving the outer vector moves the
            // inner ones, so the entries' box pointers stay valid
            ex->box_store[dir] = std::move(store);
            ex->entries[dir] = sent;
            ex->uentries[dir] = uent;
            if (receive) rent = sent;
            if (!sent.empty())
                (receive ? ex->sunpack : ex->spack) =
                    std::make_unique<splan>(sent.data(), int(sent.size()), receive ? 1 : 0);
            if (!sent.empty() && g_tune.self_tile_bytes != g_tune.tile_bytes)
            {
                // candidate plans for the fused self exchange (kept only if it is fusable)
                const uint32_t saved = g_tune.tile_bytes;
                g_tune.tile_bytes = g_tune.self_tile_bytes;
                try
                {
                    (receive ? ex->self_unpack : ex->self_pack) =
                        std::make_unique<splan>(sent.data(), int(sent.size()), receive ? 1 : 0);
                }
                catch (...)
                {
                    g_tune.tile_bytes = saved;
                    throw;
                }
                g_tune.tile_bytes = saved;
            }
            if (!uent.empty())
                (receive ? ex->uunpack : ex->upack) =
                    std::make_unique<uplan>(uent.data(), int(uent.size()), receive ? 1 : 0);
        }
        if (!ex->self_fusable() || !ex->self_pack || !ex->self_unpack ||
            !exchange_plan::same_messages(*ex->self_pack, *ex->self_unpack))
        {
            ex->self_pack.reset();
            ex->self_unpack.reset();
        }
        if (ex->self_fusable())
        {
            const splan& p = ex->self_pack ? *ex->self_pack : *ex->spack;
            const splan& q = ex->self_unpack ? *ex->self_unpack : *ex->sunpack;
            upload_pair_records(ex->self_recs, p.host_segs, q.host_segs, p.host_tiles);
        }
        build_mixed(*ex, items[0].pattern->my_rank, rent);
        *out = ex.release();
        return GHX_OK;
    });
}

int ghx_exchange_destroy(ghx_exchange* ex)
{
    return guarded([&] {
        delete ex;
        return GHX_OK;
    });
}

int ghx_exchange_num_buffers(const ghx_exchange* ex, int32_t direction, int32_t* n)
{
    return guarded([&] {
        check_ptr(ex, "exchange");
        check_ptr(n, "n");
        *n = int32_t(direction == 0 ? ex->send.size() : ex->recv.size());
        return GHX_OK;
    });
}

int ghx_exchange_buffer(const ghx_exchange* ex, int32_t direction, int32_t index,
                        int32_t* first_id, int32_t* second_id, int32_t* rank, int32_t* tag,
                        uint64_t* size)
{
    return guarded([&] {
        check_ptr(ex, "exchange");
        const auto& v = direction == 0 ? ex->send : ex->recv;
        if (index < 0 || index >= int32_t(v.size())) throw invalid("buffer index out of range");
        const auto& b = v[size_t(index)];
        if (first_id) *first_id = b.first_id;
        if (second_id) *second_id = b.second_id;
        if (rank) *rank = b.rank;
        if (tag) *tag = b.tag;
        if (size) *size = b.size;
        return GHX_OK;
    });
}

int ghx_exchange_pack(const ghx_exchange* ex, void* const* field_ptrs, int32_t n_fields,
                      void* const* send_buffers, int32_t n_send, ghx_stream stream)
{
    return guarded([&] {
        check_ptr(ex, "exchange");
        if (n_send < int32_t(ex->send.size())) throw invalid("too few send buffers");
        int rc = GHX_OK;
        if (ex->spack) rc = ex->spack->execute(field_ptrs, n_fields, send_buffers, n_send, stream);
        if (rc == GHX_OK && ex->upack)
            rc = ex->upack->execute(field_ptrs, n_fields, send_buffers, n_send, stream);
        return rc;
    });
}

int ghx_exchange_unpack(const ghx_exchange* ex, void* const* field_ptrs, int32_t n_fields,
                        void* const* recv_buffers, int32_t n_recv, ghx_stream stream)
{
    return guarded([&] {
        check_ptr(ex, "exchange");
        if (n_recv < int32_t(ex->recv.size())) throw invalid("too few recv buffers");
        int rc = GHX_OK;
        if (ex->sunpack) rc = ex->sunpack->execute(field_ptrs, n_fields, recv_buffers, n_recv, stream);
        if (rc == GHX_OK && ex->uunpack)
            rc = ex->uunpack->execute(field_ptrs, n_fields, recv_buffers, n_recv, stream);
        return rc;
    });
}

int ghx_exchange_split(ghx_exchange* ex)
{
    return guarded([&] {
        check_ptr(ex, "exchange");
        ex->make_split();
        return GHX_OK;
    });
}

int ghx_exchange_pack_buffer(const ghx_exchange* ex, int32_t index, void* const* field_ptrs,
                             int32_t n_fields, void* const* send_buffers, int32_t n_send,
                             ghx_stream stream)
{
    return guarded([&] {
        check_ptr(ex, "exchange");
        return ex->execute_buffer(0, index, field_ptrs, n_fields, send_buffers, n_send, stream);
    });
}

int ghx_exchange_unpack_buffer(const ghx_exchange* ex, int32_t index, void* const* field_ptrs,
                               int32_t n_fields, void* const* recv_buffers, int32_t n_recv,
                               ghx_stream stream)
{
    return guarded([&] {
        check_ptr(ex, "exchange");
        return ex->execute_buffer(1, index, field_ptrs, n_fields, recv_buffers, n_recv, stream);
    });
}

int ghx_exchange_self_fusable(const ghx_exchange* ex, int32_t* fusable)
{
    return guarded([&] {
        check_ptr(ex, "exchange");
        check_ptr(fusable, "fusable");
        *fusable = ex->self_fusable() ? 1 : 0;
        return GHX_OK;
    });
}

int ghx_exchange_self(const ghx_exchange* ex, void* const* field_ptrs, int32_t n_fields,
                      void* const* buffers, int32_t n_buffers, ghx_stream stream)
{
    return guarded([&] {
        check_ptr(ex, "exchange");
        if (!ex->self_fusable())
            throw invalid("exchange is not an all-self exchange with matching segments");
        const splan& p = ex->self_pack ? *ex->self_pack : *ex->spack;
        const splan& q = ex->self_unpack ? *ex->self_unpack : *ex->sunpack;
        // the launch reads the pack segments' field slots AND the unpack segments' (a domain
        // that only receives has a field slot no pack segment names, possibly the highest)
        const int nfs = std::max(p.max_field_slot, q.max_field_slot);
        if (n_fields <= nfs || n_buffers <= p.max_buf_slot)
            throw invalid("pointer arrays do not cover the plan's slots");
        if (!p.dev.segs || !q.dev.segs) throw hip_error("plan has no device tables");
        kargs a{};
        a.segs = p.dev.segs;
        a.segs2 = q.dev.segs;
        a.tile_seg = p.dev.tiles;
        a.tile_recs = ex->self_recs.recs;
        a.n_tiles = p.n_tiles;
        for (int i = 0; i <= nfs; ++i)
        {
            if (!field_ptrs[i]) throw invalid("null field pointer");
            a.field_ptr[i] = reinterpret_cast<uint64_t>(field_ptrs[i]);
        }
        for (int i = 0; i <= p.max_buf_slot; ++i)
        {
            if (!buffers[i]) throw invalid("null buffer pointer");
            a.buf_ptr[i] = reinterpret_cast<uint64_t>(buffers[i]);
        }
        return launch_self(a, stream, grid_for_tiles(p.n_tiles));
    });
}

int ghx_exchange_mixed(const ghx_exchange* ex, int32_t* mixed)
{
    return guarded([&] {
        check_ptr(ex, "exchange");
        check_ptr(mixed, "mixed");
        *mixed = ex->mixed ? 1 : 0;
        return GHX_OK;
    });
}

int ghx_exchange_pack_self(const ghx_exchange* ex, void* const* field_ptrs, int32_t n_fields,
                           void* const* send_buffers, int32_t n_send, ghx_stream stream)
{
    return guarded([&] {
        check_ptr(ex, "exchange");
        if (!ex->mixed) throw invalid("exchange has no mixed self/peer plan (ghx_exchange_mixed)");
        const splan& p = *ex->spack;
        if (n_send < int32_t(ex->send.size())) throw invalid("too few send buffers");
        // the self messages' unpack (companion) segments name receiving fields too
        const int nfs = std::max(p.max_field_slot, ex->mixed_max_field_slot);
        if (n_fields <= nfs || n_send <= p.max_buf_slot)
            throw invalid("pointer arrays do not cover the plan's slots");
        if (!p.dev.segs || !ex->mixed_comp.segs) throw hip_error("plan has no device tables");
        kargs a{};
        a.segs = p.dev.segs;
        a.segs2 = ex->mixed_comp.segs;
        a.tile_seg = p.dev.tiles;
        a.tile_recs = ex->mixed_recs.recs;
        a.n_tiles = p.n_tiles;
        for (int i = 0; i <= nfs; ++i)
        {
            if (!field_ptrs[i]) throw invalid("null field pointer");
            a.field_ptr[i] = reinterpret_cast<uint64_t>(field_ptrs[i]);
        }
        for (int i = 0; i <= p.max_buf_slot; ++i)
        {
            if (!send_buffers[i]) throw invalid("null buffer pointer");
            a.buf_ptr[i] = reinterpret_cast<uint64_t>(send_buffers[i]);
        }
        ex->mixed_parity.apply(a, {}, p.max_buf_slot + 1);
        return launch_self(a, stream, grid_for_tiles(p.n_tiles));
    });
}

int ghx_exchange_set_parity(ghx_exchange* ex, int32_t direction, const uint64_t* parity_word,
                            uint32_t parity_add, const int64_t* offsets, int32_t n_buffers)
{
    return guarded([&] {
        check_ptr(ex, "exchange");
        if (direction != 0 && direction != 1) throw invalid("direction must be 0 (pack) or 1 (unpack)");
        const size_t n = direction == 0 ? ex->send.size() : ex->recv.size();
        parity_cfg cfg;
        if (parity_word)
        {
            if (n_buffers != int32_t(n) || (n && !offsets))
                throw invalid("one offset per buffer of that direction");
            cfg.word = parity_word;
            cfg.add = parity_add & 1u;
            cfg.offset.assign(offsets, offsets + n);
            for (int64_t o : cfg.offset)
                if (o < 0 || o % 256 != 0)
                    throw invalid("second-copy offsets must be >= 0 and multiples of 256 B");
        }
        if (direction == 0)
        {
            if (ex->spack) ex->spack->parity = cfg;
            if (ex->upack) ex->upack->parity = cfg;
            ex->mixed_parity = cfg;
        }
        else
        {
            if (ex->sunpack) ex->sunpack->parity = cfg;
            if (ex->uunpack) ex->uunpack->parity = cfg;
            if (ex->punpack) ex->punpack->parity = cfg;
        }
        ex->dir_parity[direction] = cfg;
        if (ex->split) ex->set_split_parity(direction);
        return GHX_OK;
    });
}

int ghx_exchange_unpack_peers(const ghx_exchange* ex, void* const* field_ptrs, int32_t n_fields,
                              void* const* recv_buffers, int32_t n_recv, ghx_stream stream)
{
    return guarded([&] {
        check_ptr(ex, "exchange");
        if (!ex->mixed) throw invalid("exchange has no mixed self/peer plan (ghx_exchange_mixed)");
        if (n_recv < int32_t(ex->recv.size())) throw invalid("too few recv buffers");
        return ex->punpack->execute(field_ptrs, n_fields, recv_buffers, n_recv, stream);
    });
}

// ---------------------------------------------------------------------------------------------
// zero-copy put (IPC + direct field-to-field copy)
// ---------------------------------------------------------------------------------------------
int ghx_ipc_export(const void* ptr, unsigned char handle[64], uint64_t* offset)
{
    return guarded([&] {
        check_ptr(ptr, "ptr");
        check_ptr(handle, "handle");
        check_ptr(offset, "offset");
        static_assert(sizeof(hipIpcMemHandle_t) == 64, "IPC handle size");
        hipDeviceptr_t base = nullptr;
        size_t size = 0;
        if (hipMemGetAddressRange(&base, &size, const_cast<void*>(ptr)) != hipSuccess)
            throw hip_error("hipMemGetAddressRange");
        hipIpcMemHandle_t h;
        if (hipIpcGetMemHandle(&h, reinterpret_cast<void*>(base)) != hipSuccess)
        {
            char where[160];
            std::snprintf(where, sizeof(where), "hipIpcGetMemHandle (ptr %p, allocation %p + %zu B)",
                          ptr, reinterpret_cast<void*>(base), size);
            throw hip_error(where);
        }
        std::memcpy(handle, &h, sizeof(h));
        *offset = uint64_t(static_cast<const char*>(ptr) - reinterpret_cast<const char*>(base));
        return GHX_OK;
    });
}

int ghx_ipc_import(const unsigned char handle[64], uint64_t offset, void** base, void** ptr)
{
    return guarded([&] {
        check_ptr(handle, "handle");
        check_ptr(base, "base");
        check_ptr(ptr, "ptr");
        hipIpcMemHandle_t h;
        std::memcpy(&h, handle, sizeof(h));
        void* b = nullptr;
        if (hipIpcOpenMemHandle(&b, h, hipIpcMemLazyEnablePeerAccess) != hipSuccess)
            throw hip_error("hipIpcOpenMemHandle");
        *base = b;
        *ptr = static_cast<char*>(b) + offset;
        return GHX_OK;
    });
}

int ghx_ipc_close(void* base)
{
    return guarded([&] {
        check_ptr(base, "base");
        if (hipIpcCloseMemHandle(base) != hipSuccess) throw hip_error("hipIpcCloseMemHandle");
        return GHX_OK;
    });
}

int ghx_put_create(const ghx_pack_entry* src, int32_t n_src, const ghx_pack_entry* dst,
                   int32_t n_dst, ghx_put** out)
{
    return guarded([&] {
        check_ptr(out, "out");
        *out = nullptr;
        if (n_src < 0 || n_dst < 0 || (n_src && !src) || (n_dst && !dst))
            throw invalid("bad entry arrays");
        *out = new ghx_put(src, n_src, dst, n_dst);
        return GHX_OK;
    });
}

int ghx_put_execute(const ghx_put* put, void* const* src_fields, int32_t n_src,
                    void* const* dst_fields, int32_t n_dst, ghx_stream stream)
{
    return guarded([&] {
        check_ptr(put, "put");
        const splan& p = *put->from;
        const splan& q = *put->to;
        if (p.n_tiles == 0) return int(GHX_OK);
        if (n_src <= p.max_field_slot || n_dst <= q.max_field_slot)
            throw invalid("pointer arrays do not cover the plan's slots");
        if (!p.dev.segs || !q.dev.segs) throw hip_error("plan has no device tables");
        kargs a{};
        a.segs = p.dev.segs;
        a.segs2 = q.dev.segs;
        a.tile_seg = p.dev.tiles;
        a.tile_recs = put->recs.recs;
        a.n_tiles = p.n_tiles;
        for (int i = 0; i <= p.max_field_slot; ++i)
        {
            if (!src_fields[i]) throw invalid("null source field pointer");
            a.field_ptr[i] = reinterpret_cast<uint64_t>(src_fields[i]);
        }
        for (int i = 0; i <= q.max_field_slot; ++i)
        {
            if (!dst_fields[i]) throw invalid("null target field pointer");
            a.buf_ptr[i] = reinterpret_cast<uint64_t>(dst_fields[i]);
        }
        return launch_put(a, stream, grid_for_tiles(p.n_tiles));
    });
}

int ghx_put_info(const ghx_put* put, uint64_t* bytes, int32_t* n_tiles)
{
    return guarded([&] {
        check_ptr(put, "put");
        if (bytes) *bytes = put->from->bytes;
        if (n_tiles) *n_tiles = int32_t(put->from->n_tiles);
        return GHX_OK;
    });
}

int ghx_put_destroy(ghx_put* put)
{
    return guarded([&] {
        delete put;
        return GHX_OK;
    });
}

}  // extern "C"
