// ghex_amd/field_descriptor.hpp — header-only C++ adaptor: GHEX's field-descriptor concept
// (doc_src/scope/scope.rst:331-359) on top of the C ABI of libghx.so (include/ghx.h).
//
// A GHEX communication_object calls, per field and per peer buffer,
//     field.pack(T* buffer, const IndexContainer& c, void* arg)
//     field.unpack(const T* buffer, const IndexContainer& c, void* arg)
// through the std::function callbacks built in communication_object::allocate
// (include/ghex/communication_object.hpp:1007-1016) and invoked by packer<gpu>
// (include/ghex/packer.hpp:124-190), with `arg` = a cudaStream_t* / hipStream_t*.
// ghex_amd::structured::field_descriptor provides exactly that interface plus the queries
// (value_type, arch_type, dimension, layout_map, domain_id(), device_id(), num_components(),
// extents(), offsets(), byte_strides(), data()), so a communication_object-shaped caller
// drops in unchanged; every pack/unpack becomes ONE fused libghx launch for all iteration
// spaces of the container (the reference launches one kernel per iteration space,
// include/ghex/structured/pack_kernels.hpp:216-241).
//
// IndexContainer: any range of iteration-space pairs with `.local().first()[d]` and
// `.local().last()[d]` (ghex::pattern<structured grid>::iteration_space_pair,
// include/ghex/structured/pattern.hpp:95-120). Errors are thrown as std::runtime_error, the
// reference's convention (include/ghex/device/cuda/error.hpp:21-25).
//
// Depends only on <ghx.h> and the standard library; link with -lghx.
#pragma once

#include <ghx.h>

#include <array>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

namespace ghex_amd
{
inline void check(int rc, const char* what)
{
    if (rc != GHX_OK)
        throw std::runtime_error(std::string(what) + " failed: " + ghx_last_error());
}

struct gpu
{
};  // arch tag (the reference's ghex::gpu)

namespace structured
{
// Layout is given as a list of layout_map values, e.g. {2, 1, 0} for
// gridtools::layout_map<2,1,0> (dimension 0 stride-1).
template<typename T, int Dim>
class field_descriptor
{
  public:  // member types (field_descriptor.hpp:27-41)
    using value_type = T;
    using arch_type = gpu;
    using device_id_type = int;
    using domain_id_type = int;
    using coordinate_type = std::array<int, Dim>;
    using strides_type = std::array<std::int64_t, Dim>;
    static constexpr int dimension = Dim;

  private:
    domain_id_type m_dom_id;
    T* m_data;
    coordinate_type m_offsets, m_extents;
    strides_type m_byte_strides;
    std::array<int, Dim> m_layout;
    int m_num_components;
    bool m_has_components;
    device_id_type m_device;
    ghx_field_desc m_desc{};

  public:
    // wrap_field (regular/field_descriptor.hpp:167-195): offsets/extents over all Dim dims
    // (the component axis, if any, last with offset 0 and extent = num_components).
    field_descriptor(domain_id_type dom_id, T* data, const coordinate_type& offsets,
                     const coordinate_type& extents, const std::array<int, Dim>& layout,
                     int num_components = 1, bool has_components = false, int device_id = 0,
                     const strides_type* byte_strides = nullptr)
    : m_dom_id{dom_id}
    , m_data{data}
    , m_offsets{offsets}
    , m_extents{extents}
    , m_layout{layout}
    , m_num_components{num_components}
    , m_has_components{has_components}
    , m_device{device_id}
    {
        if (num_components < 1) throw std::runtime_error("number of components must be greater than 0");
        if (!has_components && num_components > 1)
            throw std::runtime_error("this field cannot have more than 1 components");
        if (byte_strides) m_byte_strides = *byte_strides;
        else
        {
            // compute_strides<D>::apply<layout,T>(extents, strides, 0) (field_utils.hpp:96-112)
            int find[Dim];
            for (int d = 0; d < Dim; ++d) find[layout[d]] = d;
            m_byte_strides[find[Dim - 1]] = sizeof(T);
            for (int k = Dim - 1; k >= 1; --k)
                m_byte_strides[find[k - 1]] = m_byte_strides[find[k]] * extents[find[k]];
        }
        m_desc.dim = Dim;
        m_desc.elem_size = int32_t(sizeof(T));
        for (int d = 0; d < Dim; ++d)
        {
            m_desc.layout[d] = layout[d];
            m_desc.byte_strides[d] = m_byte_strides[d];
            m_desc.offsets[d] = offsets[d];
            m_desc.extents[d] = extents[d];
        }
        m_desc.num_components = num_components;
        m_desc.has_components = has_components ? 1 : 0;
    }

    // queries (field_descriptor.hpp:204-226)
    device_id_type device_id() const { return m_device; }
    domain_id_type domain_id() const noexcept { return m_dom_id; }
    const coordinate_type& extents() const noexcept { return m_extents; }
    const coordinate_type& offsets() const noexcept { return m_offsets; }
    const strides_type& byte_strides() const noexcept { return m_byte_strides; }
    value_type* data() const { return m_data; }
    int num_components() const noexcept { return m_num_components; }
    const ghx_field_desc& desc() const noexcept { return m_desc; }

    // the concept's member functions (regular/field_descriptor.hpp:72-96)
    template<typename IndexContainer>
    void pack(value_type* buffer, const IndexContainer& c, void* arg)
    {
        auto boxes = to_boxes(c);
        check(ghx_structured_pack(&m_desc, m_data, buffer, boxes.data(), int32_t(boxes.size()),
                                  stream_of(arg)),
              "ghx_structured_pack");
    }

    template<typename IndexContainer>
    void unpack(const value_type* buffer, const IndexContainer& c, void* arg)
    {
        auto boxes = to_boxes(c);
        check(ghx_structured_unpack(&m_desc, m_data, buffer, boxes.data(),
                                    int32_t(boxes.size()), stream_of(arg)),
              "ghx_structured_unpack");
    }

  private:
    static constexpr int spatial() { return Dim; }

    template<typename IndexContainer>
    std::vector<ghx_box> to_boxes(const IndexContainer& c) const
    {
        std::vector<ghx_box> out;
        const int nsp = Dim - (m_has_components ? 1 : 0);
        for (const auto& is : c)
        {
            ghx_box b{};
            for (int d = 0; d < nsp; ++d)
            {
                b.first[d] = int32_t(is.local().first()[d]);
                b.last[d] = int32_t(is.local().last()[d]);
            }
            out.push_back(b);
        }
        return out;
    }

    // `arg` is a pointer to the stream handle (pack_kernels.hpp:219, 229), or nullptr.
    static ghx_stream stream_of(void* arg) { return arg ? *static_cast<ghx_stream*>(arg) : nullptr; }
};
}  // namespace structured
}  // namespace ghex_amd
