// ghx_epochs.hip — device-side access epochs for the zero-copy (bulk) exchange: the reference's
// access guards (include/ghex/rma/access_guard.hpp:35-140, shmem/access_guard.hpp) made
// stream-ordered, so that an exchange is  k_epoch(open) -> puts -> k_epoch(close)  on the caller's
// stream, with no host drain and no global barrier (include/ghex/bulk_communication_object.hpp
// :621-694 opens every target range, puts into each source range as soon as it is writable, and
// waits for its own target ranges to be written).
//
// Flag block: one POSIX shared-memory segment per node-local group of ranks, registered with the
// GPU (hipHostRegister, mapped: fine-grained, coherent host memory), so every rank's GPU reads
// and writes every rank's flags over the same physical pages. One flag per 64-B line:
//   epoch[r]    rank r's exchange counter (written by r only)
//   error[r]    set by r's kernels when a wait timed out (1: open phase, 2: close phase)
//   open[r][t]  = e: target t has opened its halos for r's puts of epoch e   (written by t)
//   done[r][s]  = e: source s's puts of epoch e into r's halos are complete (written by s)
// Exchange on rank R, epoch e = epoch[R] + 1:
//   open  (before the puts): epoch[R] = e; open[s][R] = e for every source s of R; then wait
//         until open[R][t] >= e for every target t of R (its halos are writable).
//   close (after the puts):  system-scope release; done[t][R] = e for every target t; then wait
//         until done[R][s] >= e for every source s (R's halos are written).
// Every rank runs the same number of exchanges, so the epochs agree without any reset; the
// counter lives in memory, so a captured graph replays correctly. Waits are bounded: past the
// timeout a wave records error[R] and leaves (the host reports it), so a dead peer can never
// hang the device.
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "ghx_guard.hpp"

namespace ghx
{
namespace
{
constexpr int kMaxPeers = 64;
constexpr uint64_t kMagic = 0x67687865706f6368ull;  // "ghxepoch"

struct epoch_args
{
    uint64_t* flags;  // device view of the flag block (8 uint64 per line)
    int32_t rank, world;
    int32_t n_src, n_tgt;
    uint64_t timeout_ticks;  // wall-clock ticks (hipDeviceAttributeWallClockRate kHz)
    int16_t src[kMaxPeers], tgt[kMaxPeers];
};

// line indices inside the block
__host__ __device__ inline size_t l_epoch(int r, int W) { return 1 + size_t(r) * (2 + 2 * size_t(W)); }
__host__ __device__ inline size_t l_error(int r, int W) { return l_epoch(r, W) + 1; }
__host__ __device__ inline size_t l_open(int r, int t, int W) { return l_epoch(r, W) + 2 + size_t(t); }
__host__ __device__ inline size_t l_done(int r, int s, int W) { return l_epoch(r, W) + 2 + size_t(W) + size_t(s); }
inline size_t block_lines(int W) { return 1 + size_t(W) * (2 + 2 * size_t(W)); }

__device__ __forceinline__ uint64_t* at(uint64_t* f, size_t line) { return f + line * 8; }

__device__ __forceinline__ uint64_t sys_load(uint64_t* p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void sys_store(uint64_t* p, uint64_t v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// One wave. phase 0 = open, 1 = close. Lane i signals peer i of one list and waits on peer i of
// the other; every flag address is per lane (vector memory operations only).
__global__ __launch_bounds__(64) void k_epoch(epoch_args a, int phase)
{
    const int lane = int(threadIdx.x);
    const int R = a.rank, W = a.world;
    uint64_t* f = a.flags;
    uint64_t e = sys_load(at(f, l_epoch(R, W)));
    if (phase == 0)
    {
        e += 1;
        if (lane == 0) sys_store(at(f, l_epoch(R, W)), e);
        if (lane < a.n_src) sys_store(at(f, l_open(a.src[lane], R, W)), e);  // halos open
    }
    else
    {
        // the puts of this epoch (earlier launches on this stream) before the done flags
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope
        if (lane < a.n_tgt) sys_store(at(f, l_done(a.tgt[lane], R, W)), e);
    }
    const int n = phase == 0 ? a.n_tgt : a.n_src;
    if (lane < n)
    {
        uint64_t* p = phase == 0 ? at(f, l_open(R, a.tgt[lane], W)) : at(f, l_done(R, a.src[lane], W));
        const uint64_t t0 = wall_clock64();
        while (sys_load(p) < e)
        {
            if (wall_clock64() - t0 > a.timeout_ticks)
            {
                sys_store(at(f, l_error(R, W)), uint64_t(phase + 1));
                break;
            }
            __builtin_amdgcn_s_sleep(8);
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
}
// Grid-wide system-scope fences, one wave per workgroup and kFenceGroups workgroups so that
// every XCD runs some (blocks are dealt round-robin over the 8 XCDs, each with its own L2). The
// fences in k_epoch run on ONE XCD; a peer's puts land in the target GPU's memory over xGMI, so
// the source writes back every XCD's L2 before signalling done (k_sys_release) and the target
// invalidates every XCD's L2 after its wait (k_sys_acquire), before its kernels read the halos.
constexpr int kFenceGroups = 64;

__global__ __launch_bounds__(64) void k_sys_release()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    __builtin_amdgcn_s_waitcnt(0);  // the write-back has completed before the wave ends
}

__global__ __launch_bounds__(64) void k_sys_acquire()
{
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
}
}  // namespace
}  // namespace ghx

using namespace ghx;

struct ghx_epochs
{
    std::string name;
    void* host = nullptr;  // the mapping
    size_t bytes = 0;
    bool registered = false;
    epoch_args args{};
    ~ghx_epochs()
    {
        if (registered) (void)hipHostUnregister(host);
        if (host) munmap(host, bytes);
    }
    volatile uint64_t* line(size_t l) const { return static_cast<volatile uint64_t*>(host) + l * 8; }
};

extern "C" {

int ghx_epochs_create(const char* name, int32_t create, int32_t world, int32_t rank,
                      double timeout_s, ghx_epochs** out)
{
    return guarded([&] {
        if (!name || !out) throw invalid("null argument");
        *out = nullptr;
        if (name[0] != '/' || std::strchr(name + 1, '/')) throw invalid("shm name must be \"/name\"");
        if (world < 1 || world > kMaxPeers || rank < 0 || rank >= world)
            throw invalid("world must be in [1, 64] and rank in [0, world)");
        if (!(timeout_s > 0)) throw invalid("timeout must be > 0");
        // the creating rank removes the name again if anything below fails (no stale segment)
        struct unlink_on_fail
        {
            const char* name;
            bool armed;
            ~unlink_on_fail()
            {
                if (armed) shm_unlink(name);
            }
        } cleanup{name, create != 0};
        auto ep = std::make_unique<ghx_epochs>();
        ep->name = name;
        const long page = sysconf(_SC_PAGESIZE);
        ep->bytes = (block_lines(world) * 64 + size_t(page) - 1) / size_t(page) * size_t(page);
        const int fd = shm_open(name, create ? (O_CREAT | O_EXCL | O_RDWR) : O_RDWR, 0600);
        if (fd < 0) throw invalid(std::string("shm_open(") + name + "): " + std::strerror(errno));
        if (create && ftruncate(fd, off_t(ep->bytes)) != 0)
        {
            const int err = errno;
            close(fd);
            throw invalid(std::string("ftruncate: ") + std::strerror(err));
        }
        struct stat st{};
        if (fstat(fd, &st) != 0 || size_t(st.st_size) < ep->bytes)
        {
            close(fd);
            throw invalid("shared flag block has the wrong size (world differs between ranks?)");
        }
        ep->host = mmap(nullptr, ep->bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        close(fd);
        if (ep->host == MAP_FAILED)
        {
            ep->host = nullptr;
            throw invalid(std::string("mmap: ") + std::strerror(errno));
        }
        if (create)
        {
            ep->line(0)[0] = kMagic;
            ep->line(0)[1] = uint64_t(world);
        }
        else if (ep->line(0)[0] != kMagic || ep->line(0)[1] != uint64_t(world))
            throw invalid("shared flag block not initialised by the creating rank, or another world size");
        if (hipHostRegister(ep->host, ep->bytes, hipHostRegisterMapped) != hipSuccess)
            throw hip_error("hipHostRegister(flag block)");
        ep->registered = true;
        void* dptr = nullptr;
        if (hipHostGetDevicePointer(&dptr, ep->host, 0) != hipSuccess)
            throw hip_error("hipHostGetDevicePointer(flag block)");
        int dev = 0, khz = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0)
            throw hip_error("hipDeviceGetAttribute(wall clock rate)");
        ep->args.flags = static_cast<uint64_t*>(dptr);
        ep->args.rank = rank;
        ep->args.world = world;
        ep->args.timeout_ticks = uint64_t(timeout_s * 1e3 * double(khz));
        cleanup.armed = false;
        *out = ep.release();
        return GHX_OK;
    });
}

int ghx_epochs_unlink(const char* name)
{
    return guarded([&] {
        if (!name) throw invalid("null name");
        if (shm_unlink(name) != 0) throw invalid(std::string("shm_unlink: ") + std::strerror(errno));
        return GHX_OK;
    });
}

int ghx_epochs_peers(ghx_epochs* ep, const int32_t* sources, int32_t n_sources,
                     const int32_t* targets, int32_t n_targets)
{
    return guarded([&] {
        if (!ep) throw invalid("null epochs");
        if (n_sources < 0 || n_targets < 0 || n_sources > kMaxPeers || n_targets > kMaxPeers ||
            (n_sources && !sources) || (n_targets && !targets))
            throw invalid("bad peer lists (at most 64 each)");
        for (int i = 0; i < n_sources + n_targets; ++i)
        {
            const int32_t r = i < n_sources ? sources[i] : targets[i - n_sources];
            if (r < 0 || r >= ep->args.world || r == ep->args.rank)
                throw invalid("peer rank out of range (or this rank itself)");
        }
        ep->args.n_src = n_sources;
        ep->args.n_tgt = n_targets;
        for (int i = 0; i < n_sources; ++i) ep->args.src[i] = int16_t(sources[i]);
        for (int i = 0; i < n_targets; ++i) ep->args.tgt[i] = int16_t(targets[i]);
        return GHX_OK;
    });
}

// phase 0: open (before this rank's puts), 1: close (after them; bracketed by the grid-wide
// release / acquire when this rank has targets / sources)
int ghx_epochs_enqueue(const ghx_epochs* ep, int32_t phase, ghx_stream stream)
{
    return guarded([&] {
        if (!ep) throw invalid("null epochs");
        if (phase != 0 && phase != 1) throw invalid("phase must be 0 (open) or 1 (close)");
        const auto s = static_cast<hipStream_t>(stream);
        if (phase == 1 && ep->args.n_tgt > 0)
            hipLaunchKernelGGL(k_sys_release, dim3(kFenceGroups), dim3(64), 0, s);
        hipLaunchKernelGGL(k_epoch, dim3(1), dim3(64), 0, s, ep->args, int(phase));
        if (phase == 1 && ep->args.n_src > 0)
            hipLaunchKernelGGL(k_sys_acquire, dim3(kFenceGroups), dim3(64), 0, s);
        if (hipGetLastError() != hipSuccess) throw hip_error("k_epoch launch");
        return GHX_OK;
    });
}

// *error: 0, or 1 / 2 when a wait of the open / close phase timed out (a peer never reached the
// exchange); *epoch: this rank's exchange counter. Host reads of the coherent flag block.
int ghx_epochs_status(const ghx_epochs* ep, int32_t* error, uint64_t* epoch)
{
    return guarded([&] {
        if (!ep) throw invalid("null epochs");
        const int R = ep->args.rank, W = ep->args.world;
        if (error) *error = int32_t(ep->line(l_error(R, W))[0]);
        if (epoch) *epoch = ep->line(l_epoch(R, W))[0];
        return GHX_OK;
    });
}

int ghx_epochs_destroy(ghx_epochs* ep)
{
    delete ep;
    return GHX_OK;
}

}  // extern "C"
