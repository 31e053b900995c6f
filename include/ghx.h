/*
 * ghx.h — C ABI of ghex_amd, the MI355X-native halo pack/unpack path for GHEX.
 *
 * Plain C: pointers, sizes and status codes only (no C++ or torch types cross this line).
 * The library is libghx.so (ghex_amd/lib/). Every entry point below names the reference
 * interface it replaces (paths relative to the GHEX v0.8.0 tree). INTEGRATION.md shows the
 * binding a GHEX maintainer would add on the reference side.
 *
 * Status: every function returns GHX_OK (0) or a negative ghx_status; ghx_last_error() then
 * returns a thread-local message. No exception crosses the ABI (the reference throws
 * std::runtime_error, include/ghex/device/cuda/error.hpp:21-25; the C++ adaptor in
 * include/ghex_amd/field_descriptor.hpp converts back to that convention).
 *
 * Threading: plans and patterns are immutable after creation; executing one plan from several
 * threads on distinct streams is safe. Executions are stream-ordered and asynchronous (no host
 * synchronisation inside ghx_*_execute / ghx_*_pack / ghx_*_unpack), so they can be captured
 * into a hipGraph.
 */
#ifndef GHX_H
#define GHX_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum ghx_status
{
    GHX_OK = 0,
    GHX_ERR_INVALID = -1,    /* bad argument (shape, layout, slot, alignment ...) */
    GHX_ERR_HIP = -2,        /* a HIP runtime call failed */
    GHX_ERR_NOMEM = -3,      /* host or device allocation failed */
    GHX_ERR_PATTERN = -4,    /* pattern construction failed (e.g. inconsistent halo gids) */
} ghx_status;

/* Opaque stream handle: a hipStream_t (NULL = the default stream). Kept as void* so that this
 * header needs no HIP include. Replaces the `void* arg` = cudaStream_t* of the reference's
 * field-descriptor concept (include/ghex/structured/pack_kernels.hpp:216-234). */
typedef void* ghx_stream;

#define GHX_MAX_DIM 4     /* 3 spatial dims + 1 component axis (bindings/python/src/_pyghex/structured/types.hpp:31-63) */
#define GHX_MAX_SLOTS 64  /* field / buffer pointer slots per kernel launch; a plan whose entries
                             use more is executed as one launch per group of <= 64 (any slot >= 0) */

/* Process-wide tuning knobs (development / benchmarking; defaults are the measured best):
 * "grid_cap" (max workgroups, 0 = one per tile), "tile_bytes" (buffer bytes per workgroup tile),
 * "small_tile_rows" (rows per tile of short-row structured segments; 0 = by the plan's count of
 * short rows, the default), "small_row_bytes" (rows
 * shorter than this are "short"), "order" (0 segment order, 1 short-row segments first),
 * "xcd_pair" (0|1: line-sharing short-row segment pairs dispatched in lock-step groups of 8
 * tiles, same XCD), "short_pol" (field-side cache policy of short-row segments: bit 0
 * non-temporal loads, bit 1 sc1 stores), "u_tile_rows" (rows per tile of short-row index-list
 * segments), "u_tile_bytes" (tile of index-list segments with long rows), "urun" (0|1: run path
 * for 4/8-B index-list rows), "u_run_tile_rows" (rows per tile of run-heavy index lists), "self_tile_bytes" (tile of the fused self exchange),
 * "mixed_always" (0|1: build mixed self/peer plans even without short-row self messages),
 * "tile_records" (0|1: the pack / unpack launches read one per-tile record addressed by the
 * workgroup index instead of a tile table entry and then its segment; default 1),
 * "unpack_tile_bytes" (0 = tile_bytes, the default; else the long-row tile of unpack plans, whose
 * tiles of several steps the unpack kernel then software-pipelines);
 * "fast_addr" (0|1: short-form 32-bit field addressing for segments whose extents, strides and
 * span fit it; default 1), "pack_tile_rows" / "unpack_tile_rows" (0 = by the plan's rule, the
 * default; else 64..65536 rows per tile of short-row structured segments of pack / unpack plans);
 * "reset" restores every default. Plan-shaping knobs apply to plans created afterwards. Unknown
 * keys fail with GHX_ERR_INVALID (the variants removed in round 3 are listed in
 * tools/kernel_variants_r02.hip).
 * No reference counterpart (the reference hard-codes block_dim=128, 1 element per thread:
 * include/ghex/structured/pack_kernels.hpp:211-214). */
int ghx_tune(const char* key, int32_t value);

/* Per-launch kernel durations (measurement; no reference counterpart). ghx_launch_timing(1) makes
 * every kernel launch issued afterwards BY THIS THREAD record a start and a stop event at the
 * kernel's own begin and end (hipExtLaunchKernel: the interval a rocprofv3 kernel trace reports);
 * eager launches only — never enable it around a stream capture. ghx_launch_timing_read waits for
 * the recorded launches, writes up to `cap` durations in milliseconds (launch order) to `ms`, the
 * number recorded to `*n`, and releases them; ghx_launch_timing(0) stops recording (and drops
 * unread records). */
int ghx_launch_timing(int32_t enable);
int ghx_launch_timing_read(float* ms, int32_t cap, int32_t* n);

/* Last error message of the calling thread ("" if none). */
const char* ghx_last_error(void);
/* Library version string and the offload target it was compiled for ("gfx950"). */
const char* ghx_version(void);

/* ------------------------------------------------------------------------------------------
 * Structured fields
 * ------------------------------------------------------------------------------------------ */

/* A wrapped structured field: the queries of the reference's field-descriptor concept
 * (doc_src/scope/scope.rst:331-359; include/ghex/structured/field_descriptor.hpp:27-41,
 * 152-226): dimension (incl. component axis), value size, layout_map, byte strides, offsets.
 * layout[d] = gridtools::layout_map<...>::at(d); the dim whose value is dim-1 is stride-1.
 * has_components: the last dim is the component axis of extent num_components (offset 0). */
typedef struct ghx_field_desc
{
    int32_t dim;
    int32_t elem_size;                 /* sizeof(value_type), any size >= 1 */
    int32_t layout[GHX_MAX_DIM];
    int64_t byte_strides[GHX_MAX_DIM];
    int32_t offsets[GHX_MAX_DIM];
    int32_t extents[GHX_MAX_DIM];      /* informational (bounds checks), incl. halos */
    int32_t num_components;            /* >= 1 */
    int32_t has_components;            /* 0/1 */
} ghx_field_desc;

/* One iteration space in the field's local coordinates: pattern::iteration_space_pair::local()
 * (include/ghex/structured/pattern.hpp:44-120). Only the spatial dims are given; the component
 * axis is added as [0, num_components-1] (regular/field_descriptor.hpp:131-150). */
typedef struct ghx_box
{
    int32_t first[GHX_MAX_DIM];
    int32_t last[GHX_MAX_DIM];
} ghx_box;

/* One (field, list of iteration spaces) placed into one buffer at a byte offset: the
 * communication object's field_info (include/ghex/communication_object.hpp:176-188, 1059-1065). */
typedef struct ghx_pack_entry
{
    ghx_field_desc field;
    int32_t field_slot;                /* index into field_ptrs[] at execution */
    int32_t buffer_slot;               /* index into buffer_ptrs[] at execution */
    uint64_t buffer_offset;            /* byte offset of this field's data in that buffer */
    const ghx_box* boxes;              /* iteration spaces, in pattern order */
    int32_t n_boxes;
} ghx_pack_entry;

typedef struct ghx_plan ghx_plan;

/* Build a fused pack (direction 0) or unpack (direction 1) plan over many fields, iteration
 * spaces and buffers: ONE kernel launch per execution. Replaces the per-iteration-space launch
 * loop of regular::field_descriptor::pack/unpack (include/ghex/structured/regular/field_descriptor.hpp:72-96)
 * -> serialization<gpu,L>::pack/unpack (include/ghex/structured/pack_kernels.hpp:161-248), the
 * batched pack_kernel_u of packer<gpu>::pack_u (include/ghex/packer.hpp:98-121, 192-297), and
 * packer<gpu>::pack/unpack over all buffers of communication_object::pack
 * (include/ghex/communication_object.hpp:568-597; packer.hpp:124-190).
 * The packed byte layout is bit-identical to serialization<cpu>::pack_batch. Descriptor tables
 * are uploaded to device memory here (synchronously); execution never allocates. */
int ghx_plan_create(const ghx_pack_entry* entries, int32_t n_entries, int32_t direction,
                    ghx_plan** out);
/* Enqueue the plan on `stream`: pack = buffers <- fields, unpack = fields <- buffers.
 * field_ptrs/buffer_ptrs are device pointers indexed by slot (n_field_ptrs/n_buffer_ptrs must
 * cover every slot the plan uses). */
int ghx_plan_execute(const ghx_plan* plan, void* const* field_ptrs, int32_t n_field_ptrs,
                     void* const* buffer_ptrs, int32_t n_buffer_ptrs, ghx_stream stream);
int ghx_plan_destroy(ghx_plan* plan);
/* Plan facts: total buffer bytes moved per execution, number of segments (field x iteration
 * space), number of workgroup tiles, and the largest byte offset+size touched per buffer slot. */
int ghx_plan_info(const ghx_plan* plan, uint64_t* bytes, int32_t* n_segments, int32_t* n_tiles);

/* The reference's field.pack(T* buffer, const IndexContainer& c, void* arg)
 * (include/ghex/structured/regular/field_descriptor.hpp:72-83) for ONE field: iteration spaces
 * back to back from `buffer`. Convenience form of plan_create+execute (the descriptor upload is
 * stream-ordered from a pinned staging copy; prefer a cached plan in a loop). */
int ghx_structured_pack(const ghx_field_desc* field, const void* field_data, void* buffer,
                        const ghx_box* boxes, int32_t n_boxes, ghx_stream stream);
/* field.unpack(const T* buffer, const IndexContainer& c, void* arg)
 * (include/ghex/structured/regular/field_descriptor.hpp:85-96). */
int ghx_structured_unpack(const ghx_field_desc* field, void* field_data, const void* buffer,
                          const ghx_box* boxes, int32_t n_boxes, ghx_stream stream);

/* ------------------------------------------------------------------------------------------
 * Unstructured fields (index-list gather / scatter)
 * ------------------------------------------------------------------------------------------ */

/* unstructured::data_descriptor<gpu> (include/ghex/unstructured/user_concepts.hpp:526-577):
 * value(lid, level) at values + (lid*index_stride + level*level_stride)*elem_size. */
typedef struct ghx_udata_desc
{
    int32_t elem_size;
    int32_t levels;
    int32_t levels_first;              /* buffer order: levels_first ? [i][level] : [level][i] */
    int64_t index_stride;              /* in elements */
    int64_t level_stride;              /* in elements */
} ghx_udata_desc;

typedef struct ghx_upack_entry
{
    ghx_udata_desc data;
    int32_t field_slot;
    int32_t buffer_slot;
    uint64_t buffer_offset;
    const int64_t* lids;               /* HOST array of local indices (pattern order); copied to
                                          device memory as int32 (int64 if any lid >= 2^31) */
    int64_t n_lids;
} ghx_upack_entry;

typedef struct ghx_uplan ghx_uplan;

/* The reference's data_descriptor<gpu>::pack/unpack(T* buffer, const IndexContainer& c, void*
 * stream) for ONE index list (include/ghex/unstructured/user_concepts.hpp:583-666): gather
 * values[lids[i]] (all levels, the descriptor's layout) into `buffer` / scatter back. `lids` is
 * a HOST-readable array of int32 (lid_bytes 4) or int64 (8) local indices, e.g. the pattern's
 * iteration_space::local_indices(). Plans are cached by (descriptor, list address, length); a
 * hit compares the whole list with the copy the plan was built from, so a list changed in place
 * gets a new plan. Replaced plans are freed once their last execution has completed (never with
 * a device-wide synchronisation); plans executed inside a stream capture are kept alive. */
int ghx_unstructured_pack(const ghx_udata_desc* data, const void* values, void* buffer,
                          const void* lids, int32_t lid_bytes, int64_t n_lids, ghx_stream stream);
int ghx_unstructured_unpack(const ghx_udata_desc* data, void* values, const void* buffer,
                            const void* lids, int32_t lid_bytes, int64_t n_lids, ghx_stream stream);

/* Fused unstructured pack (0) / unpack (1) plan: replaces data_descriptor<gpu>::pack/unpack
 * and the four pack/unpack_kernel_levels_{first,last} launches per neighbour
 * (include/ghex/unstructured/user_concepts.hpp:455-523, 583-666). Index lists live in
 * device memory (not managed memory as in unstructured/pattern.hpp:53-57). */
int ghx_uplan_create(const ghx_upack_entry* entries, int32_t n_entries, int32_t direction,
                     ghx_uplan** out);
int ghx_uplan_execute(const ghx_uplan* plan, void* const* field_ptrs, int32_t n_field_ptrs,
                      void* const* buffer_ptrs, int32_t n_buffer_ptrs, ghx_stream stream);
int ghx_uplan_destroy(ghx_uplan* plan);
int ghx_uplan_info(const ghx_uplan* plan, uint64_t* bytes, int32_t* n_segments, int32_t* n_tiles);

/* ------------------------------------------------------------------------------------------
 * Patterns (setup time, host only): the producers of the pack inputs.
 * ------------------------------------------------------------------------------------------ */

/* One rank's domains for pattern construction, given for ALL ranks (the reference obtains them
 * with MPI all_gather, include/ghex/structured/pattern.hpp:268-273). */
typedef struct ghx_regular_domain
{
    int32_t id;
    int32_t rank;
    int32_t first[3];
    int32_t last[3];
} ghx_regular_domain;

typedef struct ghx_pattern ghx_pattern;

/* halo_generator::operator() (include/ghex/structured/regular/halo_generator.hpp:93-148):
 * receive boxes of one domain, in the reference's order. Writes up to max_boxes boxes
 * (local first/last into `local`, global first/last into `global`), returns the count in
 * *n_boxes (call with max_boxes = 0 to query). halos = (dim0-, dim0+, dim1-, dim1+, ...). */
int ghx_regular_halo_boxes(int32_t dim, const int32_t* global_first, const int32_t* global_last,
                           const int32_t* halos, const int32_t* periodic,
                           const int32_t* domain_first, const int32_t* domain_last,
                           ghx_box* local, ghx_box* global, int32_t max_boxes, int32_t* n_boxes);

/* make_pattern<structured::grid> (include/ghex/structured/pattern.hpp:214-571), computed for
 * rank `my_rank` from all ranks' domains (ordered by rank, then each rank's d_range order). */
int ghx_regular_pattern_create(int32_t dim, const ghx_regular_domain* domains,
                               int32_t n_domains, const int32_t* global_first,
                               const int32_t* global_last, const int32_t* halos,
                               const int32_t* periodic, int32_t my_rank, ghx_pattern** out);

/* make_staged_pattern (include/ghex/structured/regular/make_pattern.hpp:47-250): `dim` pattern
 * handles written to out[0..dim-1], stage i exchanging the halos of dimension i over the domain
 * box extended by the halos of stages 0..i-1 (exchanging the stages in order fills edges and
 * corners). domains as for ghx_regular_pattern_create (all ranks); neighbors[(k*dim + i)*2 + s]
 * = the id of domain k's left (s = 0) / right (s = 1) neighbour in dimension i — the reference's
 * domain look-up `d_lu(id, offset)` evaluated for offset -1/+1 along i; only consulted where
 * that side has a halo (non-zero width, and periodic or inside the global box). */
int ghx_staged_pattern_create(int32_t dim, const ghx_regular_domain* domains, int32_t n_domains,
                              const int32_t* neighbors, const int32_t* global_first,
                              const int32_t* global_last, const int32_t* halos,
                              const int32_t* periodic, int32_t my_rank, ghx_pattern** out);

/* unstructured::domain_descriptor(id, gids, outer lids) (include/ghex/unstructured/
 * user_concepts.hpp:37-176): gids in storage order, the local ids of the outer (halo) cells.
 * Builds the gid -> lid maps (flat hash tables) once; immutable afterwards (shareable between
 * threads). Fails (GHX_ERR_PATTERN) on a repeated outer lid or a repeated inner gid, like the
 * reference's constructor. */
typedef struct ghx_udomain ghx_udomain;
int ghx_udomain_create(int32_t id, const int64_t* gids, int64_t n_gids, const int64_t* outer_lids,
                       int64_t n_outer, ghx_udomain** out);
int ghx_udomain_destroy(ghx_udomain* d);
int ghx_udomain_info(const ghx_udomain* d, int32_t* id, int64_t* size, int64_t* inner_size,
                     int64_t* n_outer);
/* halo_generator::operator() (user_concepts.hpp:234-256) as gids: the domain's reduced halo, i.e.
 * the gids of make_outer_lids(gen_gids) (n_gen < 0: all outer gids in storage order). Writes
 * *n_halo <= max(n_gen, n_outer) gids; cap must hold them. */
int ghx_udomain_halo(const ghx_udomain* d, const int64_t* gen_gids, int64_t n_gen,
                     int64_t* halo_gids, int64_t cap, int64_t* n_halo);

/* make_pattern<unstructured::grid> (include/ghex/unstructured/pattern.hpp:187-370) for ONE rank,
 * in the reference's three steps; the caller moves the bytes between ranks (only halo gids ever
 * travel, never a rank's full gid list):
 *   1. ghx_upattern_create with this rank's domains and the global max domain count per rank and
 *      max domain id (the tag layout, :218-233);
 *   2. ghx_upattern_add_halos once per rank r (this one included; any order) with r's domain ids
 *      and reduced halos (ghx_udomain_halo, concatenated): creates this rank's send halos for
 *      every halo gid that is an inner cell of one of its domains (:284-330) and a record per
 *      (my domain, r's domain) pair whose gid list must reach rank dst_rank (ghx_upattern_record:
 *      the pointer stays valid until ghx_upattern_destroy);
 *   3. ghx_upattern_add_recv for every record addressed to this rank (src = the record's sender):
 *      make_outer_lids -> receive halos (:337-365); then ghx_upattern_finish.
 * Maps are keyed and ordered (rank, tag) as the reference's (pattern.hpp:105-110). */
typedef struct ghx_upattern ghx_upattern;
int ghx_upattern_create(const ghx_udomain* const* domains, int32_t n_domains, int32_t my_rank,
                        int32_t max_num_domains, int32_t max_domain_id, ghx_upattern** out);
int ghx_upattern_add_halos(ghx_upattern* b, int32_t rank, int32_t n_domains,
                           const int32_t* domain_ids, const int64_t* halo_sizes,
                           const int64_t* halo_gids, int64_t* n_records);
int ghx_upattern_record(const ghx_upattern* b, int64_t k, int32_t* src_id, int32_t* dst_id,
                        int32_t* dst_rank, int32_t* tag, int64_t* n_gids, const int64_t** gids);
int ghx_upattern_add_recv(ghx_upattern* b, int32_t src_rank, int32_t src_id, int32_t dst_id,
                          int32_t tag, const int64_t* gids, int64_t n_gids);
int ghx_upattern_finish(ghx_upattern* b, ghx_pattern** out);
int ghx_upattern_destroy(ghx_upattern* b);

int ghx_pattern_destroy(ghx_pattern* p);
/* A copy of a pattern whose send and receive halo maps keep only the keys whose remote rank is
 * in `ranks` (keep = 1) or is not (keep = 0); tags and max_tag unchanged. The bulk exchange
 * splits a pattern this way into its node-local part (puts) and its remote part (a buffered
 * exchange), as the reference's bulk object splits it into local and remote pattern maps
 * (include/ghex/bulk_communication_object.hpp:330-383). */
int ghx_pattern_filter(const ghx_pattern* p, const int32_t* ranks, int32_t n_ranks, int32_t keep,
                       ghx_pattern** out);
/* Number of local domains (patterns) of this rank, and the global max tag
 * (pattern_container::max_tag, include/ghex/pattern_container.hpp:78-83). */
int ghx_pattern_num_domains(const ghx_pattern* p, int32_t* n);
int ghx_pattern_max_tag(const ghx_pattern* p, int32_t* max_tag);
int ghx_pattern_domain_id(const ghx_pattern* p, int32_t local_index, int32_t* id);
/* Halo maps of local domain `local_index`: direction 0 = send_halos(), 1 = recv_halos(),
 * in std::map key order. Key k: remote domain id, remote rank, tag, #iteration spaces and
 * #elements (spatial). */
int ghx_pattern_num_keys(const ghx_pattern* p, int32_t local_index, int32_t direction,
                         int32_t* n_keys);
int ghx_pattern_key(const ghx_pattern* p, int32_t local_index, int32_t direction, int32_t key,
                    int32_t* remote_id, int32_t* remote_rank, int32_t* tag, int32_t* n_spaces,
                    int64_t* n_elements);
/* Structured: the iteration spaces of a key (local and global boxes). */
int ghx_pattern_key_boxes(const ghx_pattern* p, int32_t local_index, int32_t direction,
                          int32_t key, ghx_box* local, ghx_box* global, int32_t max_boxes);
/* Unstructured: the local index list of a key (its single iteration space). */
int ghx_pattern_key_lids(const ghx_pattern* p, int32_t local_index, int32_t direction,
                         int32_t key, int64_t* lids, int64_t max_lids);

/* ------------------------------------------------------------------------------------------
 * Exchange planning: communication_object::allocate semantics (buffer per domain pair, fields
 * in exchange() order, alignof padding, tag = pattern tag + container tag offset)
 * (include/ghex/communication_object.hpp:483-566, 1003-1067).
 * ------------------------------------------------------------------------------------------ */

typedef struct ghx_exchange_item
{
    const ghx_pattern* pattern;        /* the field's pattern container (this rank) */
    int32_t local_index;               /* which local domain of that pattern */
    int32_t kind;                      /* 0 = structured (field), 1 = unstructured (udata) */
    ghx_field_desc field;              /* kind 0 */
    ghx_udata_desc udata;              /* kind 1 */
    int32_t align;                     /* alignof(value_type) */
    int32_t tag_offset;                /* prepare_exchange_buffers tag map (:540-549) */
} ghx_exchange_item;

typedef struct ghx_exchange ghx_exchange;

/* Plans one exchange() of n_items fields (field_slot = item index). Produces the send and recv
 * buffer lists (std::map order of domain_id_pair) and fused pack / unpack plans over them
 * (buffer_slot = buffer index). */
int ghx_exchange_create(const ghx_exchange_item* items, int32_t n_items, ghx_exchange** out);
int ghx_exchange_destroy(ghx_exchange* ex);
/* direction 0 = send buffers, 1 = recv buffers. */
int ghx_exchange_num_buffers(const ghx_exchange* ex, int32_t direction, int32_t* n);
int ghx_exchange_buffer(const ghx_exchange* ex, int32_t direction, int32_t index,
                        int32_t* first_id, int32_t* second_id, int32_t* rank, int32_t* tag,
                        uint64_t* size);
/* Enqueue the fused pack of all send buffers / fused unpack of all recv buffers. */
int ghx_exchange_pack(const ghx_exchange* ex, void* const* field_ptrs, int32_t n_fields,
                      void* const* send_buffers, int32_t n_send, ghx_stream stream);
int ghx_exchange_unpack(const ghx_exchange* ex, void* const* field_ptrs, int32_t n_fields,
                        void* const* recv_buffers, int32_t n_recv, ghx_stream stream);

/* Per-buffer plans: ghx_exchange_split builds one pack and one unpack plan per buffer (setup
 * time, synchronous upload); ghx_exchange_pack_buffer / ghx_exchange_unpack_buffer then enqueue
 * the pack of send buffer `index` / the unpack of recv buffer `index` alone, with the same
 * pointer arrays as ghx_exchange_pack/unpack. This is the reference's per-buffer packer call on
 * the buffer's own stream (include/ghex/communication_object.hpp:568-597, packer.hpp:124-190),
 * used to send each message as soon as its own pack is done (:611-637). */
int ghx_exchange_split(ghx_exchange* ex);
int ghx_exchange_pack_buffer(const ghx_exchange* ex, int32_t index, void* const* field_ptrs,
                             int32_t n_fields, void* const* send_buffers, int32_t n_send,
                             ghx_stream stream);
int ghx_exchange_unpack_buffer(const ghx_exchange* ex, int32_t index, void* const* field_ptrs,
                               int32_t n_fields, void* const* recv_buffers, int32_t n_recv,
                               ghx_stream stream);

/* ------------------------------------------------------------------------------------------
 * RCCL transport (one rank per GPU, xGMI inside a node): replaces oomph's NCCL backend
 * (start_group/send/recv/end_group, include/ghex/communication_object.hpp:278-281, 641-714).
 * RCCL is loaded at run time from `path` (NULL: "librccl.so.1") — pass the library the process
 * already uses (torch's), so one RCCL instance serves both.
 * ------------------------------------------------------------------------------------------ */
int ghx_rccl_open(const char* path);
int ghx_rccl_unique_id(unsigned char id[128]);
/* ncclCommInitRank (blocking until all `nranks` ranks have called it). */
int ghx_rccl_comm_init(const unsigned char id[128], int32_t nranks, int32_t rank, void** comm);
int ghx_rccl_comm_destroy(void* comm);
/* GHX_OK, or the communicator's asynchronous error as GHX_ERR_HIP. */
int ghx_rccl_comm_check(void* comm);

/* Per-peer pipelined exchange (the reference's per-buffer streams + send-as-packed,
 * include/ghex/device/cuda/stream.hpp:25-73, communication_object.hpp:568-637, 703-767): for
 * each peer, in the given order, on its own greatest-priority stream: pack of its send buffers,
 * one RCCL group {recv..., send...} on comms[k] (the peer is rank comm_ranks[k] there), unpack of
 * its recv buffers. Messages of one pair are issued in (tag, domain pair) order on both sides.
 * Peer k rides stream k mod max_streams (the device has few hardware queues, 4 by default:
 * streams beyond them share queues in an order no one chooses; dealt this way every stream
 * still runs its peers in the global order). Buffers of ranks not listed must be self messages
 * (my_rank): packed and unpacked on the
 * caller's stream. ghx_pipeline_run enqueues all of it; the caller's stream then waits for every
 * peer stream (no host synchronisation). Every rank must list its peers in one global order
 * consistent across ranks (e.g. round-robin tournament rounds) so that no wait cycle can form
 * when streams share hardware queues. Not re-entrant: one run at a time per pipeline. */
typedef struct ghx_pipeline ghx_pipeline;
int ghx_pipeline_create(ghx_exchange* ex, int32_t my_rank, int32_t n_peers,
                        const int32_t* peer_ranks, void* const* comms, const int32_t* comm_ranks,
                        int32_t max_streams, ghx_pipeline** out);
int ghx_pipeline_run(const ghx_pipeline* pl, void* const* field_ptrs, int32_t n_fields,
                     void* const* send_buffers, int32_t n_send, void* const* recv_buffers,
                     int32_t n_recv, ghx_stream stream);
int ghx_pipeline_destroy(ghx_pipeline* pl);

/* Self messages (a periodic wrap onto the same rank, or two domains of one rank) never leave
 * the device in the reference's stream-aware flow either (communication_object.hpp:703-767:
 * pack -> send to self -> unpack). When EVERY message of an exchange is a self message
 * (*fusable = 1), ghx_exchange_self performs pack and unpack in ONE launch: each workgroup packs
 * a tile of the send buffer and then writes the same bytes into the halos (from the registers it
 * stored them from, or after a workgroup barrier). The buffers are the send buffers (they double
 * as recv buffers); every packed byte and every halo byte is written, and the send buffers hold
 * the packed message afterwards. */
int ghx_exchange_self_fusable(const ghx_exchange* ex, int32_t* fusable);
int ghx_exchange_self(const ghx_exchange* ex, void* const* field_ptrs, int32_t n_fields,
                      void* const* buffers, int32_t n_buffers, ghx_stream stream);

/* Exchanges with self messages AND peer messages (*mixed = 1; e.g. a (2,1,1) periodic
 * decomposition: x to the neighbour, y and z onto the rank itself): ghx_exchange_pack_self packs
 * every send buffer AND completes the self messages (their halos written in the same launch);
 * the transport then carries the peer messages only, and ghx_exchange_unpack_peers unpacks the
 * peer recv buffers only (same pointer arrays as ghx_exchange_pack/unpack). Together they do
 * exactly what ghx_exchange_pack + ghx_exchange_unpack do. */
int ghx_exchange_mixed(const ghx_exchange* ex, int32_t* mixed);
int ghx_exchange_pack_self(const ghx_exchange* ex, void* const* field_ptrs, int32_t n_fields,
                           void* const* send_buffers, int32_t n_send, ghx_stream stream);
int ghx_exchange_unpack_peers(const ghx_exchange* ex, void* const* field_ptrs, int32_t n_fields,
                              void* const* recv_buffers, int32_t n_recv, ghx_stream stream);

/* Double-buffered buffers (the direct exchange's one-launch epochs, ghx_epochs_enqueue phase 2):
 * every later pack (direction 0: ghx_exchange_pack, _pack_self, _pack_buffer) or unpack (1:
 * ghx_exchange_unpack, _unpack_peers, _unpack_buffer) launch of `ex` uses, for buffer i with
 * offsets[i] != 0, the copy at
 * buffer_ptr + offsets[i] when (*parity_word + parity_add) is odd, read on the device at launch
 * (a captured graph alternates on replay). offsets: one per buffer of that direction, multiples
 * of 256 B (0 = one copy). parity_word = NULL restores single buffers. The reference has no
 * equivalent (its RMA path puts field to field, include/ghex/structured/rma_put.hpp:204-245). */
int ghx_exchange_set_parity(ghx_exchange* ex, int32_t direction, const uint64_t* parity_word,
                            uint32_t parity_add, const int64_t* offsets, int32_t n_buffers);

/* ------------------------------------------------------------------------------------------
 * Zero-copy put between node-local GPUs. Replaces the reference's RMA path:
 * bulk_communication_object (include/ghex/bulk_communication_object.hpp:206-704), the
 * gpu_to_gpu put (include/ghex/structured/rma_put.hpp:204-245: one launch per range, one
 * element per thread) and the CUDA IPC handles (include/ghex/rma/cuda/handle.hpp:20-96).
 * ------------------------------------------------------------------------------------------ */

/* Export the device allocation holding `ptr` for another process: a 64-byte IPC handle of the
 * allocation's base and the byte offset of `ptr` inside it (torch's caching allocator hands out
 * interior pointers). */
int ghx_ipc_export(const void* ptr, unsigned char handle[64], uint64_t* offset);
/* Map another process's allocation: *base is what ghx_ipc_close releases, *ptr = base+offset. */
int ghx_ipc_import(const unsigned char handle[64], uint64_t offset, void** base, void** ptr);
int ghx_ipc_close(void* base);

/* A put plan: src[k] and dst[k] describe the two ends of the same virtual message bytes — the
 * iteration spaces of a sender's send halo (its local coordinates, its field) and of the
 * receiver's recv halo for the same key (the receiver's coordinates and field), each entry's
 * buffer_slot/buffer_offset placing it in a virtual message exactly as ghx_plan_create would.
 * Field slots: src entries index src_fields, dst entries index dst_fields (< 64 each: one
 * launch; the bulk objects group their messages into several put plans).
 * Execution copies every element straight from the source field into the target field (peer
 * memory through ghx_ipc_import, or the same device): no buffer, one launch. Fails with
 * GHX_ERR_INVALID when the two sides do not describe the same bytes. */
typedef struct ghx_put ghx_put;
int ghx_put_create(const ghx_pack_entry* src, int32_t n_src, const ghx_pack_entry* dst,
                   int32_t n_dst, ghx_put** out);
int ghx_put_execute(const ghx_put* put, void* const* src_fields, int32_t n_src,
                    void* const* dst_fields, int32_t n_dst, ghx_stream stream);
int ghx_put_info(const ghx_put* put, uint64_t* bytes, int32_t* n_tiles);
int ghx_put_destroy(ghx_put* put);

/* Device-side access epochs of the zero-copy exchanges (bulk puts, direct pack): the reference's
 * access guards (include/ghex/rma/access_guard.hpp:35-140; per range: start/end_target_epoch on
 * the owner, start/end_source_epoch on the putter; include/ghex/bulk_communication_object.hpp
 * :621-694) as TWO stream-ordered launches around the data launch(es) — phase 0 (open) before,
 * phase 1 (close) after. The flags live in each rank's inbox, fine-grained device memory on its
 * GPU that its node-local peers map through IPC and write into, polled locally; a block of
 * node-shared host memory (POSIX shm `name`, "/...") carries the inbox handles and each rank's
 * epoch and error for the host (the creating rank passes create = 1 before the others attach
 * with 0, and one rank unlinks the name once all have attached). `world` and `rank` are the node-local group's size
 * and this rank's index in it (one block per host; at most 64 ranks per host). ghx_epochs_peers
 * (before the first ghx_epochs_enqueue; refused afterwards: enqueued kernels hold the peers'
 * inbox mappings) sets this rank's sources (ranks that write into its memory) and targets (ranks whose memory it
 * writes into) as node-local indices, excluding itself. Open: this rank's halos / receive
 * buffers are open to its sources; wait until each target has opened. Close: system-scope
 * release on every XCD (the grid is sized from the queried XCD count; the leader checks that
 * every XCD ran), signal each target, wait for each source, system-scope acquire on every XCD.
 * No host synchronisation, no barrier; the epoch counter lives in memory, so the sequence can
 * be captured into a graph. Waits are bounded: ghx_epochs_status reports 0, 1 / 2 (a wait of
 * the open / close phase timed out), 3 (the close kernel did not reach every XCD in time) or
 * 4 | s << 8 (source s failed an epoch wait: its later writes may have overlapped this rank's
 * reads). After a nonzero status the object is broken (every later wait returns at once). */
typedef struct ghx_epochs ghx_epochs;
int ghx_epochs_create(const char* name, int32_t create, int32_t world, int32_t rank,
                      double timeout_s, ghx_epochs** out);
int ghx_epochs_unlink(const char* name);
int ghx_epochs_peers(ghx_epochs* ep, const int32_t* sources, int32_t n_sources,
                     const int32_t* targets, int32_t n_targets);
int ghx_epochs_enqueue(ghx_epochs* ep, int32_t phase, ghx_stream stream);
int ghx_epochs_status(const ghx_epochs* ep, int32_t* error, uint64_t* epoch);
int ghx_epochs_info(const ghx_epochs* ep, int32_t* n_xcc, int32_t* fence_groups);
/* Phase 2 (one launch per exchange) is for receive memory double-buffered by epoch parity
 * (ghx_exchange_set_parity with the word ghx_epochs_counter returns): data launch (copy e&1 of
 * the targets') -> ghx_epochs_enqueue(ep, 2, stream) -> unpack (copy e&1 of this rank's). The
 * close tells the sources that this rank's previous unpack is done, which is what the open
 * phase is for otherwise. An object runs phases 0/1 or phase 2, not both. Without peers the
 * close phases enqueue nothing. */
int ghx_epochs_counter(const ghx_epochs* ep, const uint64_t** word);
int ghx_epochs_destroy(ghx_epochs* ep);

/* ------------------------------------------------------------------------------------------
 * Host staging copies (the NIC-side path): device <-> pinned host copies on
 * SDMA engines chosen by measurement. Replaces the staging the reference leaves to its transport
 * (oomph device/host buffers, include/ghex/arch_traits.hpp:51-75; the non-stream-aware branch of
 * include/ghex/communication_object.hpp:611-637, 715-729). hipMemcpyAsync lets the runtime pick
 * the engine, and D2H and H2D of one exchange often end up on one engine (serialised) or on a
 * slow one; ghx_copier_create probes engines 0-3 with `probe_bytes` copies per direction and
 * alone / concurrently, and keeps the pair (D2H engine, H2D engine) with the best concurrent
 * rate (ghx_copier_info). ghx_copier_submit enqueues one copy (direction 0 = device -> host,
 * 1 = host -> device; host memory must be pinned, e.g. hipHostMalloc) and returns a ticket; with
 * after_ticket >= 0 the copy engine starts it only once that earlier copy has completed (no host
 * round trip). ghx_copier_wait blocks until a ticket's copy has completed (error after
 * `timeout_s`). ghx_copier_acquire enqueues, on a stream, the cache invalidation that kernels
 * reading bytes an H2D copy has written need before them (the HIP runtime does not see these
 * copies, so it would not add it). Not thread-safe: one copier per thread. */
typedef struct ghx_copier ghx_copier;
int ghx_copier_create(uint64_t probe_bytes, double timeout_s, ghx_copier** out);
int ghx_copier_info(const ghx_copier* c, int32_t* d2h_engine, int32_t* h2d_engine, float* d2h_GBps,
                    float* h2d_GBps, float* both_GBps);
int ghx_copier_submit(ghx_copier* c, void* dst, const void* src, uint64_t bytes, int32_t direction,
                      int64_t after_ticket, uint64_t* ticket);
int ghx_copier_wait(ghx_copier* c, uint64_t ticket);
int ghx_copier_acquire(const ghx_copier* c, ghx_stream stream);
int ghx_copier_destroy(ghx_copier* c);

#ifdef __cplusplus
}
#endif

#endif /* GHX_H */
