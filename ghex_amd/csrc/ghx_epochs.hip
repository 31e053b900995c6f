// ghx_epochs.hip — device-side access epochs for the zero-copy exchanges (bulk puts, direct
// pack): the reference's access guards (include/ghex/rma/access_guard.hpp:35-140,
// shmem/access_guard.hpp) made stream-ordered:
//     puts:    k_epoch_open -> put launch(es) -> k_epoch_close      (phases 0, 1)
//     direct:  pack -> k_epoch_close1 -> unpack                     (phase 2, double buffers)
// on the caller's stream, with no host drain and no global barrier
// (include/ghex/bulk_communication_object.hpp:621-694 opens every target range, puts into each
// source range as soon as it is writable, and waits for its own target ranges to be written).
//
// Where the flags live:
//   inbox of rank R — fine-grained device memory on R's GPU (coherent across agents), IPC-mapped
//     into R's node-local peers: open[t] = e (target t opened its memory for R's writes of
//     epoch e; written by t) and done[s] = e (source s's writes of e into R's memory are complete
//     and visible; written by s). R polls only its own inbox, locally.
//   host block — one POSIX shm segment per host, indexed by node-local rank: epoch[r] and
//     error[r] for the host (ghx_epochs_status), and each rank's inbox IPC handle.
//   device words of R (plain device memory): the epoch counter and a failure mark, one
//     "written back" word per XCD, the leader's "go", an arrival count, and R's error word.
//
// Exchange on rank R, epoch e = counter + 1:
//   open  (one wave): counter = e; open[R] = e in every source's inbox; wait until every target
//         has written open[t] >= e into R's inbox (their memory is writable).
//   close (a few one-wave workgroups on EVERY XCD — the XCD count is queried, and the leader
//         checks that each XCD really ran one):
//         every workgroup: system-scope release (writes back its XCD's L2: the data launch's
//           remote writes leave every XCD's L2 for the target's memory) -> "XCD x written back";
//         leader: once every XCD has written back, done[R] = e in every target's inbox (with the
//           FAIL bit when R's own open wait failed), then wait until every source's done >= e
//           -> "go";
//         every workgroup, after "go": system-scope acquire (invalidates its XCD's L2 and its
//           CU's L1), so the kernels after the close read what the sources wrote, not stale lines.
//   close1 (phase 2): see k_epoch_close1.
// Every rank runs the same number of exchanges, so the epochs agree without any reset; the
// counters live in memory, so a captured graph replays correctly (every replay a new epoch).
// Waits are bounded: past the timeout a wave records R's error and leaves, and the host raises
// (ghx_epochs_status). A failure reaches both sides: a rank whose wait timed out (its next data
// launch may write into a target still reading that memory) marks its done flags FAIL, and every
// target that sees FAIL records error 4 with the source's index; a wait also ends as soon as an
// error is recorded for this rank.
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
constexpr int kMaxPeers = 63;  // lane 63 of a waiting wave polls the error line
constexpr int kMaxXcc = 16;    // XCC_ID is a 4-bit field
constexpr int kFencePerXcc = 4;
constexpr uint64_t kMagic = 0x67687865706f6368ull;  // "ghxepoch"
constexpr uint64_t kFail = 1ull << 63;              // done flag of a source whose open failed
// error codes (error[r]; the host decodes them in ghx_epochs_status)
constexpr uint64_t kErrOpen = 1, kErrClose = 2, kErrFence = 3, kErrPeer = 4;  // peer: 4 | s << 8

struct epoch_args
{
    uint64_t* flags;  // device view of the host block (status: epoch and error per rank)
    uint64_t* dev;    // this rank's device words (8 uint64 per line)
    uint64_t* box;    // this rank's inbox (fine-grained device memory, the peers write into it)
    int32_t rank, world;
    int32_t n_src, n_tgt;
    int32_t n_xcc;
    uint64_t timeout_ticks;  // wall-clock ticks (hipDeviceAttributeWallClockRate kHz)
    int16_t src[kMaxPeers], tgt[kMaxPeers];
    uint64_t* src_box[kMaxPeers];  // the sources' inboxes (IPC mappings; this process's own
    uint64_t* tgt_box[kMaxPeers];  // when a peer is a thread of it)
};

// host block (one per host, POSIX shm): line 0 = {magic, world}; per rank r: the epoch and the
// error for the host (ghx_epochs_status), and its inbox's IPC handle (64 B) + {offset, pid, ptr}
__host__ __device__ inline size_t l_epoch(int r, int W) { return 1 + size_t(r) * 4; }
__host__ __device__ inline size_t l_error(int r, int W) { return l_epoch(r, W) + 1; }
inline size_t l_handle(int r) { return 1 + size_t(r) * 4 + 2; }
inline size_t block_lines(int W) { return 1 + size_t(W) * 4; }
// inbox of rank R (fine-grained device memory on R's GPU; 64-B lines):
//   open[t] = e: target t has opened its halos / receive buffers for R's writes of epoch e
//   done[s] = e: source s's writes of epoch e into R's memory are complete and visible
__host__ __device__ inline size_t in_open(int t) { return size_t(t); }
__host__ __device__ inline size_t in_done(int s, int W) { return size_t(W) + size_t(s); }
inline size_t box_lines(int W) { return 2 * size_t(W); }
// device words: line 0 = {epoch counter, failure mark}, 1 + x = XCD x written back, go, the
// one-launch close's arrival count, and this rank's error (polled by its own waits)
constexpr size_t d_rel(int x) { return 1 + size_t(x); }
constexpr size_t d_go = 1 + kMaxXcc;
constexpr size_t d_arrive = d_go + 1;
constexpr size_t d_err = d_arrive + 1;
constexpr size_t kDevLines = d_err + 1;

__device__ __forceinline__ uint64_t* at(uint64_t* f, size_t line) { return f + line * 8; }

__device__ __forceinline__ uint64_t sys_load(uint64_t* p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// Flag store at system scope (sc0 sc1), relaxed: no flag of this protocol publishes data
// written by the storing wave itself. The open flags follow only reads (the stream's earlier
// kernels are done with the memory: kernel-boundary order); the done flags follow the per-XCD
// release of every workgroup of the close kernel, which the leader has observed before it
// stores them (each "XCD written back" word is stored after that XCD's buffer_wbl2 and an
// explicit wait for it).
__device__ __forceinline__ void sys_store(uint64_t* p, uint64_t v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint64_t dev_load(uint64_t* p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void dev_store(uint64_t* p, uint64_t v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ unsigned xcc_id()
{
    // HW_REG_XCC_ID (hwreg 20), bits 3:0: the XCD this wave runs on (gfx940+). The close kernels
    // use it modulo the partition's XCD count (hipDeviceAttributeNumberOfXccs): in a partitioned
    // mode (DPX/CPX) the register may report the physical XCD (e.g. 4..7 of a 4-XCD partition),
    // whose residues are still one slot per XCD. Only the unpartitioned (SPX) mode has run here.
    return __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 0xf;
}

// this rank's error: the device word its waits poll, and the host's copy (ghx_epochs_status)
__device__ __forceinline__ void record(const epoch_args& a, uint64_t code)
{
    sys_store(at(a.dev, d_err), code);
    sys_store(at(a.flags, l_error(a.rank, a.world)), code);
}

// One wave: every lane with a flag polls it (in this rank's inbox) until it reaches e (flag
// values may carry kFail); lane 63 polls this rank's error word. Returns 0 once every flag has
// arrived, the recorded error as soon as one is set, or `code` after recording it on timeout.
// *seen: the lane's last flag value (for the FAIL bit).
__device__ uint64_t wave_wait(const epoch_args& a, uint64_t* flag, uint64_t e, uint64_t code,
                              uint64_t* seen)
{
    const int lane = int(threadIdx.x);
    uint64_t* p = lane == 63 ? at(a.dev, d_err) : flag;
    const uint64_t t0 = wall_clock64();
    for (;;)
    {
        const uint64_t v = p ? sys_load(p) : 0;
        const uint64_t err = __shfl(v, 63);
        if (err) return err;
        *seen = v;
        const bool pending = lane != 63 && flag && (v & ~kFail) < e;
        if (!__any(pending)) return 0;
        if (wall_clock64() - t0 > a.timeout_ticks)
        {
            if (lane == 63) record(a, code);
            return code;
        }
        __builtin_amdgcn_s_sleep(2);
    }
}

// One wave: lanes with a device word poll it until it reaches e. False on timeout.
__device__ bool wave_wait_dev(uint64_t* word, uint64_t e, uint64_t timeout)
{
    const uint64_t t0 = wall_clock64();
    for (;;)
    {
        const uint64_t v = word ? dev_load(word) : e;
        if (!__any(v < e)) return true;
        if (wall_clock64() - t0 > timeout) return false;
        __builtin_amdgcn_s_sleep(2);
    }
}

__global__ __launch_bounds__(64) void k_epoch_open(epoch_args a)
{
    const int lane = int(threadIdx.x);
    const int R = a.rank, W = a.world;
    const uint64_t e = dev_load(at(a.dev, 0)) + 1;
    if (lane == 0)
    {
        dev_store(at(a.dev, 0), e);
        sys_store(at(a.flags, l_epoch(R, W)), e);  // the host's view (ghx_epochs_status)
    }
    if (lane < a.n_src) sys_store(at(a.src_box[lane], in_open(R)), e);  // halos / buffers open
    uint64_t seen;
    const uint64_t err = wave_wait(a, lane < a.n_tgt ? at(a.box, in_open(a.tgt[lane])) : nullptr,
                                   e, kErrOpen, &seen);
    // a failed open phase makes this epoch's done flags FAIL (the data launch runs anyway: its
    // writes may have hit memory a target was still reading, and the target must know)
    if (err && lane == 0) dev_store(at(a.dev, 0) + 1, e);
    // no fence: nothing read after this depends on the flags (the data launch that follows only
    // writes, and starts after this kernel has ended)
}

__global__ __launch_bounds__(64) void k_epoch_close(epoch_args a)
{
    const int lane = int(threadIdx.x);
    const int R = a.rank, W = a.world;
    uint64_t* dv = a.dev;
    // the data launch's writes into the targets' memory leave this XCD's L2: the write-back is
    // issued first and overlaps the loads of the epoch words; the explicit wait covers both
    if (a.n_tgt > 0) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope
    const uint64_t e = dev_load(at(dv, 0));
    const bool open_failed = dev_load(at(dv, 0) + 1) == e;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (a.n_tgt > 0 && lane == 0) dev_store(at(dv, d_rel(int(xcc_id() % unsigned(a.n_xcc)))), e);
    if (blockIdx.x == 0)
    {
        uint64_t seen = 0;
        uint64_t err = 0;
        // every XCD has written back (and the grid really reached every XCD)
        if (a.n_tgt > 0 &&
            !wave_wait_dev(lane < a.n_xcc ? at(dv, d_rel(lane)) : nullptr, e, a.timeout_ticks))
        {
            err = kErrFence;
            if (lane == 0) record(a, kErrFence);
        }
        const uint64_t mark = (open_failed || err) ? kFail : 0;
        if (lane < a.n_tgt) sys_store(at(a.tgt_box[lane], in_done(R, W)), e | mark);
        if (!err)
        {
            err = wave_wait(a, lane < a.n_src ? at(a.box, in_done(a.src[lane], W)) : nullptr, e,
                            kErrClose, &seen);
            // a source whose open failed: its writes may have overlapped this rank's last reads
            const bool bad = !err && lane < a.n_src && lane != 63 && (seen & kFail);
            const uint64_t m = __ballot(bad);
            if (m && lane == int(__builtin_ctzll(m))) record(a, kErrPeer | (uint64_t(a.src[lane]) << 8));
        }
        if (lane == 0 && a.n_src > 0) dev_store(at(dv, d_go), e);
    }
    else if (a.n_src > 0)
    {
        // the leader sets go within its own bounded waits (2 x timeout at most): a follower
        // that outlasts 3 x timeout means the leader never ran
        if (!wave_wait_dev(lane == 0 ? at(dv, d_go) : nullptr, e, 3 * a.timeout_ticks) && lane == 0)
            record(a, kErrFence);
    }
    // what the sources wrote is read by the kernels after this one: no stale line in this XCD's
    // L2 (nor this CU's L1; the next launch invalidates the other CUs' L1s). A rank without
    // sources reads nothing new and skips it.
    if (a.n_src > 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope
}
// One-launch close (phase 2) for exchanges whose receive memory is double-buffered by epoch
// parity (the direct exchange: ghx_exchange_set_parity). Epoch e = counter + 1; the data launch
// before it wrote copy e&1 of each target's buffers, the unpack after it reads copy e&1 of this
// rank's. No open phase: the copy a source writes at e+1 was last read by this rank's unpack of
// e-1, which ran before this close (stream order), so this close tells its sources so
// (open[R] = e in their inboxes) together with done[R] = e in its targets', and waits for both
// from its peers:
//   every workgroup: system-scope release (if it has targets) -> "XCD x written back"; arrive;
//   leader: every XCD written back and every workgroup arrived (all have read the counter);
//     done and open flags (done with FAIL after an earlier failure of R); wait until every
//     source's done >= e (its writes of e are in copy e&1) and every target's open >= e (it is
//     done reading the copy R writes at e+1); counter = e; go;
//   every workgroup after go: system-scope acquire.
__global__ __launch_bounds__(64) void k_epoch_close1(epoch_args a)
{
    const int lane = int(threadIdx.x);
    const int R = a.rank, W = a.world;
    uint64_t* dv = a.dev;
    if (a.n_tgt > 0) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope
    const uint64_t e = dev_load(at(dv, 0)) + 1;
    const bool failed_before = dev_load(at(dv, 0) + 1) != 0;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0)
    {
        if (a.n_tgt > 0) dev_store(at(dv, d_rel(int(xcc_id() % unsigned(a.n_xcc)))), e);
        __hip_atomic_fetch_add(at(dv, d_arrive), uint64_t(1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (blockIdx.x == 0)
    {
        uint64_t err = 0, seen = 0;
        if (a.n_tgt > 0 &&
            !wave_wait_dev(lane < a.n_xcc ? at(dv, d_rel(lane)) : nullptr, e, a.timeout_ticks))
            err = kErrFence;
        if (!err && !wave_wait_dev(lane == 0 ? at(dv, d_arrive) : nullptr, e * gridDim.x, a.timeout_ticks))
            err = kErrFence;
        if (err && lane == 0) record(a, err);
        const uint64_t mark = (failed_before || err) ? kFail : 0;
        if (lane < a.n_tgt) sys_store(at(a.tgt_box[lane], in_done(R, W)), e | mark);
        if (lane < a.n_src) sys_store(at(a.src_box[lane], in_open(R)), e);
        if (!err)
        {
            // lanes [0, n_src): the sources' done flags; [n_src, n_src + n_tgt): the targets'
            const int ns = a.n_src, nt = a.n_tgt;
            uint64_t* flag = lane < ns ? at(a.box, in_done(a.src[lane], W))
                             : lane < ns + nt ? at(a.box, in_open(a.tgt[lane - ns])) : nullptr;
            err = wave_wait(a, flag, e, kErrClose, &seen);
            const bool bad = !err && lane < ns && (seen & kFail);
            const uint64_t m = __ballot(bad);
            if (m && lane == int(__builtin_ctzll(m))) record(a, kErrPeer | (uint64_t(a.src[lane]) << 8));
        }
        if (lane == 0)
        {
            if (err) dev_store(at(dv, 0) + 1, 1);  // later done flags carry FAIL
            dev_store(at(dv, 0), e);
            dev_store(at(dv, d_go), e);
            sys_store(at(a.flags, l_epoch(R, W)), e);  // the host's view (ghx_epochs_status)
        }
    }
    else if (!wave_wait_dev(lane == 0 ? at(dv, d_go) : nullptr, e, 4 * a.timeout_ticks) && lane == 0)
        record(a, kErrFence);  // the leader never ran (its waits are bounded)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope
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
    uint64_t* dev = nullptr;
    uint64_t* box = nullptr;                 // this rank's inbox (fine-grained device memory)
    struct import_t
    {
        int rank;        // node-local rank
        void* base;      // its inbox allocation's IPC mapping (what hipIpcCloseMemHandle takes)
        uint64_t* box;   // its inbox inside that mapping
    };
    std::vector<import_t> imports;
    int fence_groups = 0;
    int mode = -1;  // 0: open + close (phases 0, 1); 1: one-launch close (phase 2)
    epoch_args args{};
    void close_imports()
    {
        for (auto& im : imports)
            if (im.base) (void)hipIpcCloseMemHandle(im.base);
        imports.clear();
    }
    ~ghx_epochs()
    {
        close_imports();
        if (box) (void)hipFree(box);
        if (dev) (void)hipFree(dev);
        if (registered) (void)hipHostUnregister(host);
        if (host) munmap(host, bytes);
    }
    // rank r's inbox in this process: its IPC mapping (or the pointer itself when r is this
    // process, e.g. two ranks as threads of one process)
    uint64_t* inbox_of(int r)
    {
        for (auto& im : imports)
            if (im.rank == r) return im.box;
        const volatile uint64_t* meta = line(l_handle(r) + 1);
        if (meta[3] != kMagic) throw invalid("a peer has not published its epoch inbox (not attached?)");
        if (int64_t(meta[1]) == int64_t(getpid())) return reinterpret_cast<uint64_t*>(meta[2]);
        hipIpcMemHandle_t h;
        std::memcpy(&h, const_cast<const uint64_t*>(line(l_handle(r))), sizeof(h));
        void* p = nullptr;
        if (hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess) != hipSuccess)
            throw hip_error("hipIpcOpenMemHandle(a peer's epoch inbox)");
        uint64_t* b = static_cast<uint64_t*>(p) + meta[0] / sizeof(uint64_t);
        imports.push_back({r, p, b});
        return b;
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
        if (world < 1 || world > kMaxPeers + 1 || rank < 0 || rank >= world)
            throw invalid("world (the node-local group) must be in [1, 64] and rank in [0, world)");
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
        int dev = 0, khz = 0, xcc = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0)
            throw hip_error("hipDeviceGetAttribute(wall clock rate)");
        // the close kernel's fences must run on every XCD (each has its own L2): its grid is
        // sized from the XCD count, and its leader checks that every XCD reported
        if (hipDeviceGetAttribute(&xcc, hipDeviceAttributeNumberOfXccs, dev) != hipSuccess || xcc < 1 ||
            xcc > kMaxXcc)
            throw hip_error("hipDeviceGetAttribute(number of XCCs) gave no usable count");
        if (hipMalloc(&ep->dev, kDevLines * 64) != hipSuccess) throw hip_error("hipMalloc(epoch words)");
        // the inbox the peers write their flags into: fine-grained device memory (coherent across
        // agents, polled locally), published to the host's other ranks through the host block
        if (hipExtMallocWithFlags(reinterpret_cast<void**>(&ep->box), box_lines(world) * 64,
                                  hipDeviceMallocFinegrained) != hipSuccess)
            throw hip_error("hipExtMallocWithFlags(epoch inbox, fine-grained)");
        if (hipMemset(ep->dev, 0, kDevLines * 64) != hipSuccess ||
            hipMemset(ep->box, 0, box_lines(world) * 64) != hipSuccess || hipDeviceSynchronize() != hipSuccess)
            throw hip_error("hipMemset(epoch words)");
        hipIpcMemHandle_t h;
        if (hipIpcGetMemHandle(&h, ep->box) != hipSuccess) throw hip_error("hipIpcGetMemHandle(epoch inbox)");
        static_assert(sizeof(h) <= 64, "IPC handle fits a line");
        std::memcpy(const_cast<uint64_t*>(ep->line(l_handle(rank))), &h, sizeof(h));
        volatile uint64_t* meta = ep->line(l_handle(rank) + 1);
        meta[0] = 0;  // offset of the inbox in its allocation
        meta[1] = uint64_t(getpid());
        meta[2] = reinterpret_cast<uint64_t>(ep->box);
        meta[3] = kMagic;  // published last
        ep->fence_groups = kFencePerXcc * xcc;
        ep->args.flags = static_cast<uint64_t*>(dptr);
        ep->args.dev = ep->dev;
        ep->args.box = ep->box;
        ep->args.rank = rank;
        ep->args.world = world;
        ep->args.n_xcc = xcc;
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
            throw invalid("bad peer lists (at most 63 each)");
        for (int i = 0; i < n_sources + n_targets; ++i)
        {
            const int32_t r = i < n_sources ? sources[i] : targets[i - n_sources];
            if (r < 0 || r >= ep->args.world || r == ep->args.rank)
                throw invalid("peer out of range of the node-local group (or this rank itself)");
        }
        // kernels already enqueued or captured hold the peers' inbox pointers by value: the
        // mappings must not change under them
        if (ep->mode >= 0)
            throw invalid("ghx_epochs_peers: peers are fixed once the epochs have been enqueued");
        // the peers' inboxes (every peer has attached: the caller's setup passed its barrier)
        ep->close_imports();
        ep->args.n_src = ep->args.n_tgt = 0;
        for (int i = 0; i < n_sources; ++i) ep->args.src_box[i] = ep->inbox_of(sources[i]);
        for (int i = 0; i < n_targets; ++i) ep->args.tgt_box[i] = ep->inbox_of(targets[i]);
        ep->args.n_src = n_sources;
        ep->args.n_tgt = n_targets;
        for (int i = 0; i < n_sources; ++i) ep->args.src[i] = int16_t(sources[i]);
        for (int i = 0; i < n_targets; ++i) ep->args.tgt[i] = int16_t(targets[i]);
        return GHX_OK;
    });
}

// phase 0: open (before this rank's data launch), 1: close (after it) — two launches per
// exchange; phase 2: the one-launch close of double-buffered exchanges (after the data launch,
// before the unpack). An object uses phases 0/1 or phase 2, never both.
int ghx_epochs_enqueue(ghx_epochs* ep, int32_t phase, ghx_stream stream)
{
    return guarded([&] {
        if (!ep) throw invalid("null epochs");
        if (phase < 0 || phase > 2) throw invalid("phase must be 0 (open), 1 (close) or 2 (one-launch close)");
        const int mode = phase == 2 ? 1 : 0;
        if (ep->mode >= 0 && ep->mode != mode)
            throw invalid("an epochs object runs either open/close (phases 0, 1) or the one-launch close (2)");
        if (phase == 2 && ep->args.n_src + ep->args.n_tgt > kMaxPeers)
            throw invalid("the one-launch close waits on at most 63 sources + targets");
        ep->mode = mode;
        const auto s = static_cast<hipStream_t>(stream);
        // no peers: nothing to close (and no double-buffered peer message reads the counter)
        if (phase != 0 && ep->args.n_src == 0 && ep->args.n_tgt == 0) return GHX_OK;
        if (phase == 0)
            hipLaunchKernelGGL(k_epoch_open, dim3(1), dim3(64), 0, s, ep->args);
        else if (phase == 1)
            hipLaunchKernelGGL(k_epoch_close, dim3(ep->fence_groups), dim3(64), 0, s, ep->args);
        else
            hipLaunchKernelGGL(k_epoch_close1, dim3(ep->fence_groups), dim3(64), 0, s, ep->args);
        if (hipGetLastError() != hipSuccess) throw hip_error("k_epoch launch");
        return GHX_OK;
    });
}

// *error: 0, 1 / 2 when a wait of the open / close phase timed out (a peer never reached the
// exchange), 3 when the close kernel's workgroups did not reach every XCD in time, 4 | s << 8
// when source s (node-local index) failed an epoch wait; *epoch: this rank's exchange
// counter. Host reads of the coherent flag block.
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

// The XCD count the close kernel was sized for and its grid.
int ghx_epochs_info(const ghx_epochs* ep, int32_t* n_xcc, int32_t* fence_groups)
{
    return guarded([&] {
        if (!ep) throw invalid("null epochs");
        if (n_xcc) *n_xcc = ep->args.n_xcc;
        if (fence_groups) *fence_groups = ep->fence_groups;
        return GHX_OK;
    });
}

// The device word holding this rank's epoch counter: the parity word of double-buffered
// launches (ghx_exchange_set_parity): a pack before the phase-2 close of epoch e reads e - 1
// (parity_add 1), an unpack after it reads e (parity_add 0).
int ghx_epochs_counter(const ghx_epochs* ep, const uint64_t** word)
{
    return guarded([&] {
        if (!ep || !word) throw invalid("null argument");
        *word = ep->dev;
        return GHX_OK;
    });
}

int ghx_epochs_destroy(ghx_epochs* ep)
{
    delete ep;
    return GHX_OK;
}

}  // extern "C"
