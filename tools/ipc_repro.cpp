// ipc_repro.cpp — developer reproducer (not product): the object-replacement IPC sequence of
// DESIGN.md §5.4 with HIP calls only (no torch, no libghx), W processes on one GPU, handles
// exchanged through a POSIX shm block with a spin barrier:
//   1. allocate A1 (bytes), fill it, export it, import every peer's A1, write a marker into each
//      peer's A1 through the mapping (hipMemcpy), barrier, check the markers peers wrote into mine
//   2. allocate A2, fill it
//   3. "teardown": close the imports of the peers' A1 and free a few small allocations (as a
//      bulk object's destruction does)
//   4. export A2, import every peer's A2, write markers, barrier, check them
// Prints one line per rank: both exports' status and the marker checks.
// Build: hipcc -O2 --offload-arch=gfx950 tools/ipc_repro.cpp -o tools/bin/ipc_repro -lrt
// Run:   tools/ipc_repro.sh [W] [MiB] [teardown 0|1]   (ipc_repro init|unlink <name>: the block)
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <unistd.h>

#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace
{
constexpr int kMaxW = 16;
struct shared
{
    std::atomic<int> arrived[64];
    hipIpcMemHandle_t h[2][kMaxW];
    int export_rc[2][kMaxW];
    hipIpcMemHandle_t hb[2][kMaxW];  // the fine-grained "inbox" of each round (inbox mode)
    int inbox_rc[2][kMaxW];
};

shared* g = nullptr;
int W = 4, R = 0;

void barrier(int k)
{
    g->arrived[k].fetch_add(1);
    while (g->arrived[k].load() < W) usleep(50);
}

// write marker (round * 100 + me) into the first 8 bytes of slot `me` of every peer's block;
// each rank then checks the slots of its own block
void write_markers(const std::vector<void*>& peer, int round)
{
    for (int r = 0; r < W; ++r)
    {
        if (r == R || !peer[size_t(r)]) continue;
        const uint64_t v = uint64_t(round) * 100 + uint64_t(R);
        (void)hipMemcpy(static_cast<char*>(peer[size_t(r)]) + 4096 * R, &v, 8, hipMemcpyHostToDevice);
    }
    (void)hipDeviceSynchronize();
}

int check_markers(void* mine, int round)
{
    int bad = 0;
    for (int r = 0; r < W; ++r)
    {
        if (r == R) continue;
        uint64_t v = 0;
        (void)hipMemcpy(&v, static_cast<char*>(mine) + 4096 * r, 8, hipMemcpyDeviceToHost);
        if (v != uint64_t(round) * 100 + uint64_t(r)) ++bad;
    }
    return bad;
}
}  // namespace

int main(int argc, char** argv)
{
    if (argc > 2 && (!std::strcmp(argv[1], "init") || !std::strcmp(argv[1], "unlink")))
    {
        if (!std::strcmp(argv[1], "unlink")) return shm_unlink(argv[2]) == 0 ? 0 : 5;
        const int f = shm_open(argv[2], O_CREAT | O_RDWR | O_TRUNC, 0600);
        if (f < 0 || ftruncate(f, sizeof(shared)) != 0) return 6;
        void* m = mmap(nullptr, sizeof(shared), PROT_READ | PROT_WRITE, MAP_SHARED, f, 0);
        if (m == MAP_FAILED) return 7;
        std::memset(m, 0, sizeof(shared));
        return 0;
    }
    W = argc > 1 ? std::atoi(argv[1]) : 4;
    R = argc > 2 ? std::atoi(argv[2]) : 0;
    const size_t bytes = size_t(argc > 3 ? std::atoi(argv[3]) : 136) << 20;
    const int teardown = argc > 4 ? std::atoi(argv[4]) : 1;
    const char* name = argc > 5 ? argv[5] : "/ghx_ipc_repro";
    // 1: each round also exports a small fine-grained allocation (as the epochs' inbox), imports
    // the peers' and, at the teardown, closes them and frees its own
    const int inbox = argc > 6 ? std::atoi(argv[6]) : 0;
    if (W < 2 || W > kMaxW) return 2;
    int fd = shm_open(name, O_RDWR, 0600);
    if (fd < 0) return 3;
    g = static_cast<shared*>(mmap(nullptr, sizeof(shared), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0));
    if (g == MAP_FAILED) return 4;
    (void)hipSetDevice(0);
    void* a[2] = {nullptr, nullptr};
    std::vector<void*> peer(size_t(W), nullptr);
    int bad[2] = {0, 0}, import_fail[2] = {0, 0};
    std::vector<void*> small, boxes;
    void* box[2] = {nullptr, nullptr};
    for (int round = 0; round < 2; ++round)
    {
        if (round == 0 || a[1] == nullptr)
        {
            (void)hipMalloc(&a[round], bytes);
            (void)hipMemset(a[round], 0, bytes);
            (void)hipDeviceSynchronize();
        }
        if (round == 0)
        {
            // step 2 happens before the teardown: A2 allocated while round 0's imports live
            for (int i = 0; i < 4; ++i)
            {
                void* p = nullptr;
                (void)hipMalloc(&p, 65536);
                small.push_back(p);
            }
        }
        g->export_rc[round][R] = int(hipIpcGetMemHandle(&g->h[round][R], a[round]));
        if (inbox)
        {
            (void)hipExtMallocWithFlags(&box[round], 4096, hipDeviceMallocFinegrained);
            (void)hipMemset(box[round], 0, 4096);
            (void)hipDeviceSynchronize();
            g->inbox_rc[round][R] = int(hipIpcGetMemHandle(&g->hb[round][R], box[round]));
        }
        barrier(4 * round + 0);
        if (inbox)
            for (int r = 0; r < W; ++r)
            {
                if (r == R || g->inbox_rc[round][r] != 0) continue;
                void* q = nullptr;
                if (hipIpcOpenMemHandle(&q, g->hb[round][r], hipIpcMemLazyEnablePeerAccess) == hipSuccess)
                    boxes.push_back(q);
            }
        for (int r = 0; r < W; ++r)
        {
            if (r == R || g->export_rc[round][r] != 0) continue;
            if (hipIpcOpenMemHandle(&peer[size_t(r)], g->h[round][r], hipIpcMemLazyEnablePeerAccess) != hipSuccess)
            {
                peer[size_t(r)] = nullptr;
                ++import_fail[round];
            }
        }
        barrier(4 * round + 1);
        write_markers(peer, round + 1);
        barrier(4 * round + 2);
        bad[round] = check_markers(a[round], round + 1);
        if (round == 0)
        {
            (void)hipMalloc(&a[1], bytes);  // A2, before the teardown
            (void)hipMemset(a[1], 0, bytes);
            (void)hipDeviceSynchronize();
            if (teardown)
            {
                for (auto& p : peer)
                    if (p) (void)hipIpcCloseMemHandle(p);
                for (void* p : small) (void)hipFree(p);
                for (void* q : boxes) (void)hipIpcCloseMemHandle(q);
                boxes.clear();
                if (box[0]) (void)hipFree(box[0]);
            }
            for (auto& p : peer) p = nullptr;
        }
        // no barrier between a rank's teardown and its next export (as in the bulk objects:
        // a peer may still be tearing down while this rank exports)
    }
    std::printf("rank %d W %d MiB %zu teardown %d inbox %d: export A1 rc %d A2 rc %d, import failures "
                "%d / %d, wrong markers A1 %d A2 %d\n",
                R, W, bytes >> 20, teardown, inbox, g->export_rc[0][R], g->export_rc[1][R],
                import_fail[0], import_fail[1], bad[0], bad[1]);
    return 0;
}
