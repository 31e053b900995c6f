"""The C++ communication object (include/ghex_amd/communication_object.hpp): the reference's
host-side exchange API (context, make_pattern, pattern(field), exchange(...).wait()) in C++ over
the C ABI, with the loopback transport (ranks as threads on one GPU) and the RCCL transport
(ncclSend/ncclRecv). Every halo cell is checked against the reference tests' self-validating
encodings (test/structured/regular/test_regular_domain.cpp:739-800: wrapped global coordinate;
test/unstructured/unstructured_test_case.hpp:345-388: dom*10000 + gid*100 + level)."""
import json
import os
import subprocess
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "cpp", "bin", "co_demo")
INC = os.path.join(ROOT, "include")
LIB = os.path.join(ROOT, "ghex_amd", "lib")


def _run(args, timeout=120):
    assert os.path.exists(EXE), "build() compiles tests/cpp/bin/co_demo"
    p = subprocess.run([EXE] + [str(a) for a in args], capture_output=True, text=True,
                       timeout=timeout)
    lines = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]
    return p.returncode, lines, p.stderr


def test_co_header_compiles_host_only(tmp_path):
    """The header set is plain host C++ (g++, HIP runtime API headers only)."""
    src = tmp_path / "t.cpp"
    src.write_text(
        '#include <ghex_amd/communication_object.hpp>\n'
        '#include <ghex_amd/field_descriptor.hpp>\n'
        'int main(){ ghex_amd::loopback_hub hub(2); ghex_amd::loopback_transport t(hub, 1);\n'
        '  ghex_amd::context ctx(t); ghex_amd::communication_options o; o.fuse_self = false;\n'
        '  return (ctx.rank() == 1 && ctx.size() == 2 && !o.fuse_self) ? 0 : 1; }\n')
    exe = tmp_path / "t"
    subprocess.run(["g++", "-std=c++17", "-D__HIP_PLATFORM_AMD__", "-I", INC, "-I",
                    "/opt/rocm/include", str(src), "-o", str(exe), "-L", LIB, "-lghx",
                    "-L/opt/rocm/lib", "-lamdhip64", f"-Wl,-rpath,{LIB}",
                    "-Wl,-rpath,/opt/rocm/lib"], check=True)
    assert subprocess.run([str(exe)]).returncode == 0


def test_co_loopback_all_gather_cpu(tmp_path):
    """make_pattern's setup collective: the loopback all_gather with threads, no GPU."""
    src = tmp_path / "g.cpp"
    src.write_text(
        '#include <ghex_amd/transport.hpp>\n#include <thread>\n'
        'int main(){ const int n = 5; ghex_amd::loopback_hub hub(n); int bad = 0;\n'
        '  std::vector<std::thread> th; for (int r = 0; r < n; ++r) th.emplace_back([&, r]{\n'
        '    ghex_amd::loopback_transport t(hub, r);\n'
        '    for (int round = 0; round < 50; ++round) {\n'
        '      std::vector<char> mine(std::size_t(r + round % 3), char(r * 7 + round));\n'
        '      auto all = t.all_gather(mine);\n'
        '      for (int q = 0; q < n; ++q) { if (all[q].size() != std::size_t(q + round % 3)) ++bad;\n'
        '        for (char c : all[q]) if (c != char(q * 7 + round)) ++bad; } } });\n'
        '  for (auto& t : th) t.join(); return bad ? 1 : 0; }\n')
    exe = tmp_path / "g"
    subprocess.run(["g++", "-std=c++17", "-pthread", "-D__HIP_PLATFORM_AMD__", "-I", INC, "-I",
                    "/opt/rocm/include", str(src), "-o", str(exe), "-L/opt/rocm/lib", "-lamdhip64",
                    "-Wl,-rpath,/opt/rocm/lib"], check=True)
    assert subprocess.run([str(exe)], timeout=60).returncode == 0


def test_co_unstructured_make_pattern_compiles_known_answer_cpu(tmp_path, golden_dir):
    """The C++ make_pattern<unstructured> (reduced halos through the transport's all_gather) on
    4 loopback threads, no GPU: every rank's send/recv lid tables equal the reference's
    known-answer tables (unstructured_test_case.hpp:217-343)."""
    import json
    with open(os.path.join(golden_dir, "unstructured_case.json")) as fh:
        case = json.load(fh)
    doms, exp = [], []
    for r in range(4):
        d = case["domains"][str(r)]
        doms.append("{%s}, {%s}" % (",".join(map(str, d["gids"])), ",".join(map(str, d["halo_lids"]))))
        for direction, key in ((0, "send_maps"), (1, "recv_maps")):
            for rid, lids in sorted(case[key][str(r)].items(), key=lambda kv: int(kv[0])):
                exp.append("{%d,%d,%s,{%s}}" % (r, direction, rid, ",".join(map(str, lids))))
    src = tmp_path / "u.cpp"
    src.write_text(
        '#include <ghex_amd/communication_object.hpp>\n#include <thread>\n#include <map>\n'
        'namespace U = ghex_amd::unstructured;\n'
        'struct E { int r, dir, rid; std::vector<long> lids; };\n'
        'int main(){ std::vector<std::pair<std::vector<long>, std::vector<long>>> doms = {'
        + ",".join("{%s}" % d for d in doms) + '};\n'
        '  std::vector<E> exp = {' + ",".join(exp) + '};\n'
        '  ghex_amd::loopback_hub hub(4); int bad = 0; std::mutex m;\n'
        '  std::vector<std::thread> th; for (int r = 0; r < 4; ++r) th.emplace_back([&, r]{\n'
        '    ghex_amd::loopback_transport t(hub, r); ghex_amd::context ctx(t);\n'
        '    U::domain_descriptor d(r, doms[r].first, doms[r].second);\n'
        '    auto pc = U::make_pattern(ctx, {}, {d});\n'
        '    std::map<std::pair<int,int>, std::vector<long>> got;\n'
        '    for (int dir = 0; dir < 2; ++dir) { int32_t nk = 0; ghx_pattern_num_keys(pc.handle(), 0, dir, &nk);\n'
        '      for (int k = 0; k < nk; ++k) { int32_t rid, rr, tag, ns; int64_t ne;\n'
        '        ghx_pattern_key(pc.handle(), 0, dir, k, &rid, &rr, &tag, &ns, &ne);\n'
        '        std::vector<long> l(ne); ghx_pattern_key_lids(pc.handle(), 0, dir, k, l.data(), ne);\n'
        '        got[{dir, rid}] = l; } }\n'
        '    std::lock_guard<std::mutex> g(m); std::size_t n = 0;\n'
        '    for (auto& e : exp) if (e.r == r) { ++n; if (got[{e.dir, e.rid}] != e.lids) ++bad; }\n'
        '    if (n != got.size()) ++bad; });\n'
        '  for (auto& t : th) t.join(); return bad ? 1 : 0; }\n')
    exe = tmp_path / "u"
    subprocess.run(["g++", "-std=c++17", "-pthread", "-D__HIP_PLATFORM_AMD__", "-I", INC, "-I",
                    "/opt/rocm/include", str(src), "-o", str(exe), "-L", LIB, "-lghx",
                    "-L/opt/rocm/lib", "-lamdhip64", f"-Wl,-rpath,{LIB}",
                    "-Wl,-rpath,/opt/rocm/lib"], check=True)
    assert subprocess.run([str(exe)], timeout=60).returncode == 0


@pytest.mark.gpu
@pytest.mark.parametrize("parts,N,H", [((1, 1, 1), 12, 2), ((2, 1, 1), 10, 2),
                                       ((2, 2, 1), 9, 1), ((2, 2, 2), 8, 3),
                                       ((3, 1, 2), 7, 2),
                                       # x-local: self messages hold the x rows -> mixed plans
                                       ((1, 1, 2), 10, 2), ((1, 2, 2), 9, 3)])
def test_co_loopback_structured(parts, N, H):
    """PX*PY*PZ ranks (threads) each with one N^3 domain and a double + a float field in one
    exchange (mixed alignment pads), two exchanges (plan reuse); every cell of every rank."""
    rc, lines, err = _run(["loopback", *parts, N, H])
    ranks = [l for l in lines if l.get("mode") == "structured"]
    assert rc == 0, (lines, err)
    assert len(ranks) == parts[0] * parts[1] * parts[2]
    assert all(l["bad"] == 0 and l["plans"] == 1 for l in ranks)


@pytest.mark.gpu
def test_co_loopback_config3_geometry():
    """BASELINE config 3's decomposition (2x2x2 periodic, 7 peers per rank: 8 MiB faces, 64 KiB
    edges, 512 B corners at 512^3) as 8 thread-ranks on one GPU at 256^3 per rank (512^3 per
    rank also passes: `co_demo loopback 2 2 2 512 2`); every cell of every rank."""
    rc, lines, err = _run(["loopback", 2, 2, 2, 256, 2], timeout=300)
    ranks = [l for l in lines if l.get("mode") == "structured"]
    assert rc == 0, (lines, err)
    assert len(ranks) == 8 and all(l["bad"] == 0 for l in ranks)


@pytest.mark.gpu
@pytest.mark.parametrize("self_through", [0, 1])
def test_co_rccl_single_rank(self_through):
    """RCCL transport: with SELF=1 the 26 self messages travel through ncclSend/ncclRecv to self
    inside one group (the rccl_transport code path on one GPU); SELF=0 the fused self launch."""
    rc, lines, err = _run(["rccl", 12, 2, self_through])
    assert rc == 0, (lines, err)
    assert [l["bad"] for l in lines if l.get("mode") == "structured"] == [0]


@pytest.mark.gpu
@pytest.mark.parametrize("levels", [1, 3])
def test_co_loopback_unstructured_known_answer(tmp_path, levels):
    """The reference's 4-domain unstructured case (unstructured_test_case.hpp:35-86), one domain
    per rank (threads), data_descriptor levels_first: every halo value = its owner's encoding."""
    case = json.load(open(os.path.join(ROOT, "tests", "golden", "unstructured_case.json")))
    f = tmp_path / "doms.txt"
    with open(f, "w") as fh:
        for i in sorted(case["domains"], key=int):
            d = case["domains"][i]
            fh.write(" ".join(str(x) for x in [i, len(d["gids"]), *d["gids"], len(d["halo_lids"]),
                                               *d["halo_lids"]]) + "\n")
    rc, lines, err = _run(["unstructured", str(f), levels])
    assert rc == 0, (lines, err)
    ranks = [l for l in lines if l.get("mode") == "unstructured"]
    assert len(ranks) == 4 and all(l["bad"] == 0 for l in ranks)


@pytest.mark.gpu
@pytest.mark.parametrize("parts,N,H", [((2, 1, 1), 10, 2), ((2, 2, 2), 8, 3), ((3, 1, 2), 7, 2),
                                       ((1, 1, 2), 10, 2)])
def test_co_loopback_pipelined(parts, N, H):
    """options.pipelined: every rank's peers in the global round order over 4 lanes, each peer
    packed / exchanged (transport::exchange_peer) / unpacked on its lane; every cell."""
    rc, lines, err = _run(["pipeloop", *parts, N, H])
    ranks = [l for l in lines if l.get("mode") == "structured"]
    assert rc == 0, (lines, err)
    assert len(ranks) == parts[0] * parts[1] * parts[2]
    assert all(l["bad"] == 0 for l in ranks)


@pytest.mark.gpu
@pytest.mark.parametrize("self_tr", [0, 1])
def test_co_rccl_pipelined(self_tr):
    """The pipelined form over the RCCL transport (one rank; self messages through
    ncclSend/ncclRecv when self_tr)."""
    rc, lines, err = _run(["rccl", 12, 2, self_tr, 1])
    assert rc == 0, (lines, err)
    assert all(l.get("bad", 1) == 0 for l in lines if l.get("mode") == "structured")


@pytest.mark.gpu
@pytest.mark.parametrize("parts,N,H", [((1, 1, 1), 12, 2), ((2, 1, 1), 10, 2), ((2, 2, 2), 8, 3),
                                       ((3, 1, 2), 7, 2), ((1, 2, 2), 9, 1)])
def test_co_bulk_loopback(parts, N, H):
    """The C++ bulk_communication_object (zero-copy puts, include/ghex_amd/
    bulk_communication_object.hpp): ranks as threads, two fields (double, float) registered
    with add_field, init, two exchanges; every cell of every rank."""
    rc, lines, err = _run(["bulkloop", *parts, N, H])
    ranks = [l for l in lines if l.get("mode") == "bulk"]
    assert rc == 0, (lines, err)
    assert len(ranks) == parts[0] * parts[1] * parts[2]
    assert all(l["bad"] == 0 and l["puts"] >= 1 and l["plans"] == 0 for l in ranks)


@pytest.mark.gpu
@pytest.mark.parametrize("parts,hosts", [((2, 2, 1), 2), ((2, 2, 2), 2), ((2, 2, 2), 4)])
def test_co_bulk_emulated_hosts(parts, hosts):
    """The C++ bulk object with its ranks spread over emulated hosts: node-local halos by puts,
    the others through the remote part (the pattern filtered to other hosts' ranks, a
    communication_object over the loopback transport), one exchange()/wait(); every cell."""
    rc, lines, err = _run(["bulkhosts", *parts, 6, 2, hosts])
    ranks = [l for l in lines if l.get("mode") == "bulk"]
    assert rc == 0, (lines, err)
    assert len(ranks) == parts[0] * parts[1] * parts[2]
    assert all(l["bad"] == 0 and l["remote"] == 1 for l in ranks)


def test_bulk_header_compiles_host_only(tmp_path):
    """The bulk header is plain host C++ too."""
    src = tmp_path / "b.cpp"
    src.write_text(
        '#include <ghex_amd/bulk_communication_object.hpp>\n'
        '#include <ghex_amd/field_descriptor.hpp>\n'
        'int main(){ ghex_amd::bulk_handle h; h.wait(); return h.is_ready() ? 0 : 1; }\n')
    exe = tmp_path / "b"
    subprocess.run(["g++", "-std=c++17", "-D__HIP_PLATFORM_AMD__", "-I", INC, "-I",
                    "/opt/rocm/include", str(src), "-o", str(exe), "-L", LIB, "-lghx",
                    "-L/opt/rocm/lib", "-lamdhip64", f"-Wl,-rpath,{LIB}",
                    "-Wl,-rpath,/opt/rocm/lib"], check=True)
    assert subprocess.run([str(exe)]).returncode == 0


@pytest.mark.gpu
@pytest.mark.parametrize("n", [2, 4])
def test_co_bulk_reference_local_rma_geometry(n):
    """test/structured/regular/test_local_rma.cpp's simulation_1 through the C++ bulk object:
    two domains per rank (self puts between them), fields with offset 3 > halo 2, double /
    float / int fields registered in the reference's order; halos filled, beyond untouched."""
    rc, lines, err = _run(["rma", n])
    ranks = [l for l in lines if l.get("mode") == "rma"]
    assert rc == 0, (lines, err)
    assert len(ranks) == n and all(l["bad"] == 0 and l["puts"] >= 1 for l in ranks)


def _run_procs(args_of_rank, n, timeout=120):
    """One co_demo process per rank (shm transport); every process's lines and exit status.
    A process still running at the timeout is killed with the rest (no rank outlives the test)."""
    assert os.path.exists(EXE), "build() compiles tests/cpp/bin/co_demo"
    procs = [subprocess.Popen([EXE] + [str(a) for a in args_of_rank(r)], stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True) for r in range(n)]
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=timeout))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    lines = [json.loads(l) for o, _ in outs for l in o.splitlines() if l.startswith("{")]
    return [p.returncode for p in procs], lines, "".join(e for _, e in outs)


def _shm_name(tag):
    return f"/ghxt_{tag}_{os.getpid()}"


@pytest.mark.parametrize("n", [2, 3, 5])
def test_shm_transport_all_gather_processes_cpu(n):
    """tests/cpp/shm_transport.hpp's setup collective with ranks as PROCESSES (no GPU
    calls): 60 all_gather rounds of varying sizes (0..4 KB) with barriers between, every byte of
    every contribution checked on every rank; the segment is unlinked once all have attached."""
    name = _shm_name(f"g{n}")
    rcs, lines, err = _run_procs(lambda r: ["shmgather", name, r, n, 60], n, timeout=60)
    assert rcs == [0] * n, (lines, err)
    assert sorted(l["rank"] for l in lines) == list(range(n))
    assert all(l["bad"] == 0 for l in lines)
    assert not os.path.exists("/dev/shm" + name)


@pytest.mark.gpu
@pytest.mark.parametrize("mode,parts,N,H", [("plain", (2, 1, 1), 10, 2), ("plain", (2, 2, 1), 9, 1),
                                            ("plain", (1, 1, 2), 10, 2), ("pipe", (2, 2, 1), 8, 2),
                                            ("pipe", (3, 1, 1), 7, 3), ("direct", (2, 1, 1), 10, 2),
                                            ("direct", (2, 2, 1), 8, 3), ("direct", (1, 1, 2), 9, 1),
                                            ("direct", (2, 2, 2), 6, 2)])
def test_co_shm_processes(mode, parts, N, H):
    """The C++ communication_object with one PROCESS per rank (shm transport, host-staged
    messages): one group or per-peer lanes; or direct (options.direct: the pack writes into the
    receivers' buffers over IPC, device epochs, no transport step); two fields (double + float:
    mixed pads), two exchanges; every cell of every rank."""
    n = parts[0] * parts[1] * parts[2]
    name = _shm_name(f"{mode}{n}")
    rcs, lines, err = _run_procs(lambda r: ["shm", name, r, *parts, N, H, mode], n)
    ranks = [l for l in lines if l.get("mode") == "structured"]
    assert rcs == [0] * n, (lines, err)
    assert len(ranks) == n and all(l["bad"] == 0 for l in ranks)


@pytest.mark.gpu
@pytest.mark.parametrize("parts,N,H,hosts", [((2, 1, 1), 10, 2, 0), ((2, 2, 1), 8, 2, 0),
                                             ((2, 2, 2), 6, 3, 0), ((2, 2, 1), 8, 2, 2),
                                             ((2, 2, 2), 6, 2, 2)])
def test_co_bulk_device_epochs_processes(parts, N, H, hosts):
    """The C++ bulk object's device-epoch form (the one it takes when every rank of a host is
    its own process): IPC puts into the other processes' halos, k_epoch open/close on the
    object's stream, no host barrier; with emulated hosts the other hosts' halos go through the
    remote part (a communication_object over the shm transport) in the same exchange().
    Every cell of every rank, two exchanges; every rank reports device epochs."""
    n = parts[0] * parts[1] * parts[2]
    name = _shm_name(f"bulk{n}h{hosts}")
    rcs, lines, err = _run_procs(lambda r: ["shm", name, r, *parts, N, H, "bulk", hosts], n)
    ranks = [l for l in lines if l.get("mode") == "bulk"]
    assert rcs == [0] * n, (lines, err)
    assert len(ranks) == n
    assert all(l["bad"] == 0 and l["epochs"] == 1 and l["puts"] >= 1 for l in ranks)
    assert all(l["remote"] == (1 if hosts else 0) for l in ranks)


def test_shm_transport_missing_peer_times_out_cpu():
    """Every wait of the shm transport is bounded: a rank whose peers never start reports an
    error naming the stage instead of hanging; rank 0 alone leaves no segment behind."""
    name = _shm_name("lonely")
    t0 = time.time()
    rc, lines, err = _run(["shmgather", name, 1, 2, 3, 1.5], timeout=30)
    assert rc == 2 and "attach" in lines[-1]["error"], (lines, err)
    rc, lines, err = _run(["shmgather", name, 0, 2, 3, 1.5], timeout=30)
    assert rc == 2 and "barrier" in lines[-1]["error"], (lines, err)
    assert time.time() - t0 < 20
    assert not os.path.exists("/dev/shm" + name)
