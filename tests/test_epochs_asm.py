"""CPU: the cross-GPU ordering of the zero-copy exchanges, pinned in the gfx950 machine code
(VERDICT r03 next #3a). The one-GPU test box cannot exercise writes that land in another chip's
HBM over xGMI, so what makes them safe is checked where it lives — the instructions hipcc emits
for the epoch kernels (ghex_amd/csrc/ghx_epochs.hip) and for the kernels that write peer memory
(k_copy: the direct exchange's pack; k_put: the bulk puts; ghex_amd/csrc/ghx_kernels.hip):

* every system-scope release (`buffer_wbl2 sc0 sc1`) is followed at once by a wait for it
  (`s_waitcnt vmcnt(0)`), so no flag store can overtake the write-back;
* the close kernel reads the XCD id (placement is checked, not assumed), releases before it
  publishes "this XCD is written back", and ends in a system-scope acquire (`buffer_inv sc0 sc1`)
  behind a wait (ranks with sources; nothing touches memory after it); the open kernel, whose
  flags follow reads only, has no fence;
* every flag access (the inboxes in fine-grained device memory, the host block) is a
  system-scope vector access (`sc0 sc1`), every device word an agent-scope one (`sc1`), none
  through `flat_` instructions;
* the peer-writing kernels store through `global_store_*` (no `flat_`, no non-temporal stores
  whose write-back the release would not cover).
Reference: include/ghex/rma/cuda/handle.hpp:20-96 (the CUDA IPC path these replace)."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"
pytestmark = pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not present")


def _asm(src, tmp_path):
    out = tmp_path / (os.path.basename(src) + ".s")
    subprocess.run([HIPCC, "-std=c++17", "-O3", "-I" + os.path.join(ROOT, "include"),
                    "-I" + os.path.join(ROOT, "ghex_amd", "csrc"), "--offload-arch=gfx950",
                    "--cuda-device-only", "-S", src, "-o", str(out)],
                   check=True, capture_output=True, timeout=600)
    return out.read_text()


def _kernels(text, name):
    """The instruction lines of every kernel whose symbol contains `name` (label to
    .Lfunc_end), comments and assembler markers dropped."""
    out = []
    for m in re.finditer(r"^(_Z\w*" + name + r"\w*):", text, re.M):
        body = text[m.end():text.index(".Lfunc_end", m.end())]
        lines = []
        for l in body.splitlines():
            l = l.split(";")[0].strip()
            if l and not l.startswith(".") and not l.endswith(":"):
                lines.append(l)
        out.append(lines)
    assert out, f"no kernel {name}"
    return out


@pytest.fixture(scope="module")
def epochs_asm(tmp_path_factory):
    return _asm(os.path.join(ROOT, "ghex_amd", "csrc", "ghx_epochs.hip"),
                tmp_path_factory.mktemp("asm"))


def _full_wait(line):
    """An s_waitcnt that waits for every outstanding vector-memory operation."""
    return re.match(r"s_waitcnt\b.*\bvmcnt\(0\)", line) is not None


def _releases_are_waited(lines):
    """Every buffer_wbl2 is system scope and a full `s_waitcnt vmcnt(0)` comes after it before
    the next store (loads may overlap the write-back; no flag store can overtake it)."""
    n = 0
    for i, l in enumerate(lines):
        if l.startswith("buffer_wbl2"):
            assert l == "buffer_wbl2 sc0 sc1", l  # system scope
            j = next(k for k in range(i + 1, len(lines)) if lines[k].startswith("global_store"))
            assert any(_full_wait(l) for l in lines[i + 1:j]), lines[i:j + 1]
            n += 1
    return n


@pytest.mark.parametrize("close", ["k_epoch_closeE", "k_epoch_close1"])
def test_every_release_is_waited_for(epochs_asm, close):
    (lines,) = _kernels(epochs_asm, close)
    assert _releases_are_waited(lines) >= 1
    # the open kernel publishes no data (its flags follow reads only): no fences at all
    (lines,) = _kernels(epochs_asm, "k_epoch_open")
    assert not [l for l in lines if l.startswith(("buffer_wbl2", "buffer_inv"))]


@pytest.mark.parametrize("close", ["k_epoch_closeE", "k_epoch_close1"])
def test_close_kernel_fences_every_xcd(epochs_asm, close):
    (lines,) = _kernels(epochs_asm, close)
    text = "\n".join(lines)
    assert "hwreg(HW_REG_XCC_ID" in text
    # the first memory write of every workgroup ("XCD x written back") comes after the
    # system-scope release and its wait
    first_rel = lines.index("buffer_wbl2 sc0 sc1")
    first_store = next(i for i, l in enumerate(lines) if l.startswith("global_store"))
    assert first_rel < first_store
    assert any(_full_wait(l) for l in lines[first_rel:first_store])
    # every system-scope acquire sits behind a full wait and ends its path (the next
    # instruction is s_endpgm: nothing touches memory after it); the one-launch close ends every
    # path with it, the two-launch close those of ranks with sources
    invs = [i for i, l in enumerate(lines) if l.startswith("buffer_inv")]
    assert invs
    for i in invs:
        assert lines[i] == "buffer_inv sc0 sc1" and _full_wait(lines[i - 1]), lines[i - 3:i + 1]
        assert lines[i + 1] == "s_endpgm", lines[i:i + 3]
    if close == "k_epoch_close1":
        ends = [i for i, l in enumerate(lines) if l == "s_endpgm"]
        assert all(lines[i - 1] == "buffer_inv sc0 sc1" for i in ends)


@pytest.mark.parametrize("kernel", ["k_epoch_open", "k_epoch_closeE", "k_epoch_close1"])
def test_flag_accesses_are_scoped_vector_ops(epochs_asm, kernel):
    (lines,) = _kernels(epochs_asm, kernel)
    mem = [l for l in lines if re.match(r"(global|flat|buffer)_(load|store|atomic)", l)]
    assert not [l for l in mem if l.startswith("flat_")]
    # the one-launch close's arrival count: a 64-bit agent-scope atomic add (as the compiler
    # lowers it for gfx950)
    atomics = [l for l in mem if l.startswith("global_atomic")]
    assert all(l.startswith("global_atomic_add_x2") for l in atomics), atomics
    mem = [l for l in mem if l not in atomics]
    # every store is a flag or word store, at system (`sc0 sc1`) or agent (`sc1`) scope
    stores = [l for l in mem if "_store" in l]
    assert stores and all(l.endswith(" sc1") for l in stores), [l for l in stores if not l.endswith(" sc1")]
    # every load either polls a flag or word (`sc1` / `sc0 sc1`) or reads the kernel arguments
    # (the peer lists and the peers' inbox pointers: plain loads of the read-only kernarg
    # segment, 16-bit ranks and 64-bit pointers)
    loads = [l for l in mem if "_load" in l]
    polls = [l for l in loads if l.endswith(" sc1")]
    plain = [l for l in loads if l not in polls]
    assert any(l.endswith(" sc0 sc1") for l in polls) and any(l.endswith(" sc1") for l in polls)
    assert all(re.match(r"global_load_(ushort|dwordx2) ", l) and " sc" not in l for l in plain), plain
    assert any(l.endswith(" sc0 sc1") for l in stores)


@pytest.fixture(scope="module")
def kernels_asm(tmp_path_factory):
    return _asm(os.path.join(ROOT, "ghex_amd", "csrc", "ghx_kernels.hip"),
                tmp_path_factory.mktemp("asmk"))


@pytest.mark.parametrize("kernel", ["k_copy", "k_put"])
def test_peer_writing_kernels_store_through_global_ops(kernels_asm, kernel):
    bodies = _kernels(kernels_asm, kernel)
    for lines in bodies:
        stores = [l for l in lines if re.match(r"(global|flat|buffer)_store", l)]
        assert stores
        assert all(l.startswith("global_store") for l in stores), stores[:4]
        assert not [l for l in stores if " nt" in l], "non-temporal peer stores"
