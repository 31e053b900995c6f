// cpol_bench.hip — developer micro-benchmark: x-normal faces of a 516^3 fp64 field at halo 2
// (2 x 512 x 512 rows of 16 B, pitch 4128 B) packed / unpacked with buffer loads / stores whose
// cache-policy bits vary on the FIELD side (gfx950: sc0 = 1, nt = 2, sc1 = 16). Question: does
// any policy turn the 16-B row accesses into smaller fabric requests or otherwise speed them up?
// Build: hipcc -O3 --offload-arch=gfx950 tools/cpol_bench.hip -o tools/bin/cpol_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                \
    do                                                                                       \
    {                                                                                        \
        hipError_t e = (x);                                                                  \
        if (e != hipSuccess)                                                                 \
        {                                                                                    \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);                  \
            exit(1);                                                                         \
        }                                                                                    \
    } while (0)

using v4 = unsigned __attribute__((ext_vector_type(4)));
constexpr int N = 512, H = 2, E = N + 2 * H;
constexpr unsigned SY = E * 8u, SZ = E * E * 8u;
constexpr unsigned ROWS = N * N;  // per face

__device__ __forceinline__ unsigned row_off(unsigned i)  // i over 2 faces
{
    const unsigned face = i / ROWS, j = i % ROWS;
    const unsigned y = j % N, z = j / N;
    return (z + H) * SZ + (y + H) * SY + (face ? N * 8u : H * 8u);
}

template<int AUX, bool PACK>
__global__ __launch_bounds__(256) void k(char* field, unsigned fbytes, char* buf)
{
    const __amdgpu_buffer_rsrc_t rf = __builtin_amdgcn_make_buffer_rsrc(field, 0, fbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(buf, 0, 2 * ROWS * 16, 0x00020000);
    constexpr int U = 4;
    const unsigned base = blockIdx.x * 256 * U + threadIdx.x;
    v4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
    {
        const unsigned i = base + u * 256;
        if (PACK) v[u] = __builtin_amdgcn_raw_buffer_load_b128(rf, row_off(i), 0, AUX);
        else v[u] = __builtin_amdgcn_raw_buffer_load_b128(rb, i * 16, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
    {
        const unsigned i = base + u * 256;
        if (PACK) __builtin_amdgcn_raw_buffer_store_b128(v[u], rb, i * 16, 0, 0);
        else __builtin_amdgcn_raw_buffer_store_b128(v[u], rf, row_off(i) - 16, 0, AUX);
    }
}

__global__ void touch(char* p, long n)
{
    for (long i = (long(blockIdx.x) * 256 + threadIdx.x) * 16; i < n; i += long(gridDim.x) * 256 * 16)
        *(v4*)(p + i) = v4{1, 2, 3, 4};
}

template<int AUX>
void run(char* f, unsigned fbytes, char* buf, char* flush, long flush_bytes, hipEvent_t e0, hipEvent_t e1)
{
    const unsigned grid = 2 * ROWS / (256 * 4);
    for (int cold = 0; cold < 2; ++cold)
    {
        float us[2] = {0, 0};
        const int reps = 20;
        for (int d = 0; d < 2; ++d)
            for (int r = 0; r < reps + 2; ++r)
            {
                if (cold) hipLaunchKernelGGL(touch, dim3(4096), dim3(256), 0, 0, flush, flush_bytes);
                CK(hipEventRecord(e0));
                if (d == 0) hipLaunchKernelGGL((k<AUX, true>), dim3(grid), dim3(256), 0, 0, f, fbytes, buf);
                else hipLaunchKernelGGL((k<AUX, false>), dim3(grid), dim3(256), 0, 0, f, fbytes, buf);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (r >= 2) us[d] += ms * 1000.f / reps;
            }
        printf("{\"aux\":%d,\"cold\":%d,\"pack_us\":%.2f,\"unpack_us\":%.2f}\n", AUX, cold, us[0], us[1]);
    }
}

int main(int argc, char** argv)
{
    const unsigned fbytes = SZ * E;
    char *f, *buf, *flush;
    CK(hipMalloc(&f, fbytes));
    CK(hipMalloc(&buf, 2 * ROWS * 16));
    const long flush_bytes = 1l << 30;
    CK(hipMalloc(&flush, flush_bytes));
    CK(hipMemset(f, 0, fbytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int only = argc > 1 ? atoi(argv[1]) : -1;
    if (only < 0 || only == 0) run<0>(f, fbytes, buf, flush, flush_bytes, e0, e1);
    if (only < 0 || only == 1) run<1>(f, fbytes, buf, flush, flush_bytes, e0, e1);
    if (only < 0 || only == 2) run<2>(f, fbytes, buf, flush, flush_bytes, e0, e1);
    if (only < 0 || only == 3) run<3>(f, fbytes, buf, flush, flush_bytes, e0, e1);
    if (only < 0 || only == 16) run<16>(f, fbytes, buf, flush, flush_bytes, e0, e1);
    if (only < 0 || only == 17) run<17>(f, fbytes, buf, flush, flush_bytes, e0, e1);
    if (only < 0 || only == 18) run<18>(f, fbytes, buf, flush, flush_bytes, e0, e1);
    if (only < 0 || only == 19) run<19>(f, fbytes, buf, flush, flush_bytes, e0, e1);
    return 0;
}
