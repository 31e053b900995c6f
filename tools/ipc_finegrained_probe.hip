// ipc_finegrained_probe.hip — can a fine-grained device allocation (hipExtMallocWithFlags,
// hipDeviceMallocFinegrained) be exported through IPC and written by another process's kernel,
// with the owner's kernel seeing the value through system-scope polls? (Developer probe before
// moving the epoch flags from pinned host memory into the receivers' device memory.)
//   ipc_finegrained_probe owner <file>   allocate, export the handle to <file>, poll for 42
//   ipc_finegrained_probe writer <file>  import the handle from <file>, store 42 from a kernel
// One JSON line from the owner. Build: make -C tools bin/ipc_finegrained_probe.
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>

#define CK(x)                                                                                  \
    do                                                                                         \
    {                                                                                          \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess)                                                                  \
        {                                                                                      \
            std::printf("{\"tool\": \"ipc_finegrained_probe\", \"ok\": false, \"error\": \"%s at line %d\"}\n", \
                        hipGetErrorString(e_), __LINE__);                                      \
            std::exit(1);                                                                      \
        }                                                                                      \
    } while (0)

__global__ void k_wait(uint64_t* p, uint64_t want, uint64_t timeout, uint64_t* out)
{
    const uint64_t t0 = wall_clock64();
    uint64_t v = 0;
    while ((v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) != want)
        if (wall_clock64() - t0 > timeout) break;
    out[0] = v;
    out[1] = wall_clock64() - t0;
}

__global__ void k_store(uint64_t* p, uint64_t v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

int main(int argc, char** argv)
{
    if (argc < 3) return 2;
    const bool owner = std::strcmp(argv[1], "owner") == 0;
    const char* file = argv[2];
    if (owner)
    {
        uint64_t* buf = nullptr;
        CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&buf), 4096, hipDeviceMallocFinegrained));
        CK(hipMemset(buf, 0, 4096));
        hipIpcMemHandle_t h;
        CK(hipIpcGetMemHandle(&h, buf));
        FILE* f = std::fopen(file, "wb");
        std::fwrite(&h, sizeof(h), 1, f);
        std::fclose(f);
        uint64_t* out = nullptr;
        CK(hipMalloc(&out, 16));
        int khz = 0;
        CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
        hipLaunchKernelGGL(k_wait, dim3(1), dim3(64), 0, 0, buf + 8, uint64_t(42), uint64_t(khz) * 20000ull, out);
        CK(hipDeviceSynchronize());
        uint64_t r[2];
        CK(hipMemcpy(r, out, 16, hipMemcpyDeviceToHost));
        std::printf("{\"tool\": \"ipc_finegrained_probe\", \"ok\": %s, \"seen\": %llu, \"wait_ms\": %.3f}\n",
                    r[0] == 42 ? "true" : "false", (unsigned long long)r[0], double(r[1]) / khz);
        std::remove(file);
        return r[0] == 42 ? 0 : 1;
    }
    hipIpcMemHandle_t h;
    FILE* f = nullptr;
    for (int i = 0; i < 200 && !f; ++i)
    {
        f = std::fopen(file, "rb");
        if (!f) std::this_thread::sleep_for(std::chrono::milliseconds(50));
    }
    if (!f) return 3;
    std::this_thread::sleep_for(std::chrono::milliseconds(200));  // the owner's write completes
    if (std::fread(&h, sizeof(h), 1, f) != 1) return 4;
    std::fclose(f);
    void* p = nullptr;
    CK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
    hipLaunchKernelGGL(k_store, dim3(1), dim3(1), 0, 0, static_cast<uint64_t*>(p) + 8, uint64_t(42));
    CK(hipDeviceSynchronize());
    CK(hipIpcCloseMemHandle(p));
    return 0;
}
