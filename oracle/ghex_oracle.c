/*
 * ghex_oracle.c — TEST INFRASTRUCTURE ONLY (the parity oracle and the CPU baseline).
 *
 * A plain-C restatement of the reference's CPU serializer for the halo
 * pack/unpack hot path. Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library; the product (ghex_amd/, libghx.so)
 * never links, loads or calls it, and has no CPU fallback.
 *
 * Restated reference functions (paths relative to the GHEX v0.8.0 tree):
 *   - serialization<cpu,Layout>::pack_batch / unpack_batch
 *       include/ghex/structured/pack_kernels.hpp:62-158
 *     one memcpy per contiguous row; rows enumerated with ghex::for_loop in
 *     layout order (include/ghex/util/for_each.hpp:85-149).
 *   - serialization<cpu,Layout>::pack / unpack (element-wise)
 *       include/ghex/structured/pack_kernels.hpp:42-60
 *   - pack_iteration_space::buffer()/data() addressing
 *       include/ghex/structured/field_descriptor.hpp:76-99, 113-136
 *   - regular::field_descriptor::pack/unpack (iteration spaces back to back)
 *       include/ghex/structured/regular/field_descriptor.hpp:72-96
 *   - make_buffer_desc (dense buffer box, strides in field layout order)
 *       include/ghex/structured/regular/field_descriptor.hpp:114-129
 *       + detail::compute_strides include/ghex/structured/field_utils.hpp:82-112
 *   - unstructured data_descriptor<cpu>::get / set
 *       include/ghex/unstructured/user_concepts.hpp:385-440
 *
 * Parity pinning: see oracle/README.md and DESIGN.md §Oracle. The halo
 * generator / pattern half of the oracle lives in oracle/oracle.py.
 *
 * Conventions: D <= 4 dimensions (3 spatial + 1 component axis, as the
 * reference's Python bindings allow, bindings/python/src/_pyghex/structured/types.hpp:31-63).
 * layout[d] is gridtools::layout_map<...>::at(d): the dimension whose layout
 * value is D-1 is the stride-1 ("contiguous") dimension.
 * A box is int32 first[D], last[D] in the field's local coordinates
 * (0 = first owned cell); data address = data + sum((x+offset)*byte_stride).
 */
#include <stdint.h>
#include <string.h>

#define ORC_MAXD 4

static int find_dim(const int32_t* layout, int D, int value)
{
    for (int d = 0; d < D; ++d)
        if (layout[d] == value) return d;
    return -1;
}

/* Byte strides of the dense buffer box, compute_strides<D>::apply<layout,T>(ext, strides, 0)
 * (field_utils.hpp:96-112): stride(find(D-1)) = s, stride(find(k-1)) = stride(find(k))*ext(find(k)). */
static void buffer_strides(int D, const int32_t* layout, const int64_t* ext, int64_t elem,
                           int64_t* bs)
{
    int idx = find_dim(layout, D, D - 1);
    bs[idx] = elem;
    for (int k = D - 1; k >= 1; --k)
    {
        int last_idx = find_dim(layout, D, k);
        int i2 = find_dim(layout, D, k - 1);
        bs[i2] = bs[last_idx] * ext[last_idx];
    }
}

typedef struct
{
    int D;
    int64_t elem;
    int32_t layout[ORC_MAXD];
    int64_t fstride[ORC_MAXD];
    int32_t offset[ORC_MAXD];
} orc_field;

/* One iteration space, row-wise (pack_batch / unpack_batch). dir 0 = pack, 1 = unpack.
 * Returns the number of bytes of buffer consumed. */
static int64_t batch_is(const orc_field* f, char* field, char* buf, const int32_t* first,
                        const int32_t* last, int dir)
{
    const int D = f->D;
    int64_t ext[ORC_MAXD] = {0}, bs[ORC_MAXD] = {0};
    int64_t n = 1;
    for (int d = 0; d < D; ++d)
    {
        ext[d] = (int64_t)last[d] - first[d] + 1;
        n *= ext[d];
    }
    if (n <= 0) return 0;
    buffer_strides(D, f->layout, ext, f->elem, bs);
    const int cont = find_dim(f->layout, D, D - 1);
    const int64_t row_bytes = ext[cont] * f->elem;
    /* loop order: layout value 0 outermost ... value D-2 innermost (for_loop over the reduced
     * layout map, pack_kernels.hpp:85-107); the contiguous dim is the memcpy. */
    int order[ORC_MAXD];
    int no = 0;
    for (int v = 0; v < D; ++v)
    {
        int d = find_dim(f->layout, D, v);
        if (d != cont) order[no++] = d;
    }
    int32_t x[ORC_MAXD];
    for (int d = 0; d < D; ++d) x[d] = first[d];
    /* the innermost loop of the nest (layout value D-2) runs with pointer increments, as the
     * reference's compile-time for_loop lets the compiler do; the outer ones as an odometer.
     * Same rows in the same order (tools/cpu_serializer_ab.cpp: 1.15-1.2x faster than
     * recomputing every row's offsets, profiles/r06_cpu_ab.jsonl). */
    const int in = no > 0 ? order[no - 1] : -1;
    const int64_t n_in = in >= 0 ? ext[in] : 1;
    const int64_t fs_in = in >= 0 ? f->fstride[in] : 0, bs_in = in >= 0 ? bs[in] : 0;
    const size_t rb = (size_t)row_bytes;
    for (;;)
    {
        int64_t foff = 0, boff = 0;
        for (int d = 0; d < D; ++d)
        {
            foff += ((int64_t)x[d] + f->offset[d]) * f->fstride[d];
            boff += ((int64_t)x[d] - first[d]) * bs[d];
        }
        char* fp = field + foff;
        char* bp = buf + boff;
        if (dir == 0)
            for (int64_t i = 0; i < n_in; ++i, fp += fs_in, bp += bs_in) memcpy(bp, fp, rb);
        else
            for (int64_t i = 0; i < n_in; ++i, fp += fs_in, bp += bs_in) memcpy(fp, bp, rb);
        /* advance the odometer over the outer dims, order[no-2] fastest */
        int k = no - 2;
        for (; k >= 0; --k)
        {
            int d = order[k];
            if (++x[d] <= last[d]) break;
            x[d] = first[d];
        }
        if (k < 0) break;
    }
    return n * f->elem;
}

/* Element-wise variant (serialization<cpu>::pack/unpack, pack_kernels.hpp:42-60): per element
 * buffer(x) = data(x). Identical bytes to batch_is whenever the contiguous dim's byte stride is
 * the element size; differs (correctly follows the strides) otherwise. */
static int64_t elementwise_is(const orc_field* f, char* field, char* buf, const int32_t* first,
                              const int32_t* last, int dir)
{
    const int D = f->D;
    int64_t ext[ORC_MAXD] = {0}, bs[ORC_MAXD] = {0};
    int64_t n = 1;
    for (int d = 0; d < D; ++d)
    {
        ext[d] = (int64_t)last[d] - first[d] + 1;
        n *= ext[d];
    }
    if (n <= 0) return 0;
    buffer_strides(D, f->layout, ext, f->elem, bs);
    int order[ORC_MAXD];
    for (int v = 0; v < D; ++v) order[v] = find_dim(f->layout, D, v);
    int32_t x[ORC_MAXD];
    for (int d = 0; d < D; ++d) x[d] = first[d];
    for (;;)
    {
        int64_t foff = 0, boff = 0;
        for (int d = 0; d < D; ++d)
        {
            foff += ((int64_t)x[d] + f->offset[d]) * f->fstride[d];
            boff += ((int64_t)x[d] - first[d]) * bs[d];
        }
        if (dir == 0) memcpy(buf + boff, field + foff, (size_t)f->elem);
        else memcpy(field + foff, buf + boff, (size_t)f->elem);
        int k = D - 1;
        for (; k >= 0; --k)
        {
            int d = order[k];
            if (++x[d] <= last[d]) break;
            x[d] = first[d];
        }
        if (k < 0) break;
    }
    return n * f->elem;
}

static void load_field(orc_field* f, int D, int64_t elem, const int32_t* layout,
                       const int64_t* byte_strides, const int32_t* offsets)
{
    f->D = D;
    f->elem = elem;
    for (int d = 0; d < D; ++d)
    {
        f->layout[d] = layout[d];
        f->fstride[d] = byte_strides[d];
        f->offset[d] = offsets[d];
    }
}

/* regular::field_descriptor::pack (field_descriptor.hpp:72-83): iteration spaces back to back.
 * boxes: n_boxes * (first[D], last[D]) int32, already expanded with the component axis.
 * mode 0 = pack_batch (row memcpy, what field_descriptor::pack calls), 1 = element-wise.
 * Returns total bytes written to the buffer. */
int64_t orc_structured_pack(const void* field, void* buffer, int D, int64_t elem,
                            const int32_t* layout, const int64_t* byte_strides,
                            const int32_t* offsets, const int32_t* boxes, int n_boxes, int mode)
{
    orc_field f;
    load_field(&f, D, elem, layout, byte_strides, offsets);
    char* b = (char*)buffer;
    int64_t total = 0;
    for (int i = 0; i < n_boxes; ++i)
    {
        const int32_t* first = boxes + (int64_t)i * 2 * D;
        const int32_t* last = first + D;
        int64_t nb = mode == 0 ? batch_is(&f, (char*)field, b, first, last, 0)
                               : elementwise_is(&f, (char*)field, b, first, last, 0);
        b += nb;
        total += nb;
    }
    return total;
}

int64_t orc_structured_unpack(void* field, const void* buffer, int D, int64_t elem,
                              const int32_t* layout, const int64_t* byte_strides,
                              const int32_t* offsets, const int32_t* boxes, int n_boxes,
                              int mode)
{
    orc_field f;
    load_field(&f, D, elem, layout, byte_strides, offsets);
    char* b = (char*)buffer;
    int64_t total = 0;
    for (int i = 0; i < n_boxes; ++i)
    {
        const int32_t* first = boxes + (int64_t)i * 2 * D;
        const int32_t* last = first + D;
        int64_t nb = mode == 0 ? batch_is(&f, (char*)field, b, first, last, 1)
                               : elementwise_is(&f, (char*)field, b, first, last, 1);
        b += nb;
        total += nb;
    }
    return total;
}

/* unstructured data_descriptor<cpu>::get (user_concepts.hpp:416-440) for one iteration space.
 * Field address of (lid, level) = values + (lid*index_stride + level*level_stride)*elem
 * (user_concepts.hpp:363-378). levels_first: buffer[i*levels + l]; else buffer[l*n + i]. */
int64_t orc_unstructured_get(const void* values, void* buffer, int64_t elem, const int64_t* lids,
                             int64_t n, int64_t levels, int levels_first, int64_t index_stride,
                             int64_t level_stride)
{
    const char* v = (const char*)values;
    char* b = (char*)buffer;
    if (levels_first)
    {
        for (int64_t i = 0; i < n; ++i)
            for (int64_t l = 0; l < levels; ++l)
            {
                memcpy(b, v + (lids[i] * index_stride + l * level_stride) * elem, (size_t)elem);
                b += elem;
            }
    }
    else
    {
        for (int64_t l = 0; l < levels; ++l)
            for (int64_t i = 0; i < n; ++i)
            {
                memcpy(b, v + (lids[i] * index_stride + l * level_stride) * elem, (size_t)elem);
                b += elem;
            }
    }
    return n * levels * elem;
}

/* unstructured data_descriptor<cpu>::set (user_concepts.hpp:385-409). */
int64_t orc_unstructured_set(void* values, const void* buffer, int64_t elem, const int64_t* lids,
                             int64_t n, int64_t levels, int levels_first, int64_t index_stride,
                             int64_t level_stride)
{
    char* v = (char*)values;
    const char* b = (const char*)buffer;
    if (levels_first)
    {
        for (int64_t i = 0; i < n; ++i)
            for (int64_t l = 0; l < levels; ++l)
            {
                memcpy(v + (lids[i] * index_stride + l * level_stride) * elem, b, (size_t)elem);
                b += elem;
            }
    }
    else
    {
        for (int64_t l = 0; l < levels; ++l)
            for (int64_t i = 0; i < n; ++i)
            {
                memcpy(v + (lids[i] * index_stride + l * level_stride) * elem, b, (size_t)elem);
                b += elem;
            }
    }
    return n * levels * elem;
}

/* FNV-1a 64 over a byte range: the size-independent checksum used for full-size parity. */
uint64_t orc_fnv1a64(const void* data, int64_t n, uint64_t h)
{
    const unsigned char* p = (const unsigned char*)data;
    if (h == 0) h = 1469598103934665603ULL;
    for (int64_t i = 0; i < n; ++i)
    {
        h ^= p[i];
        h *= 1099511628211ULL;
    }
    return h;
}
