"""The C++ drop-in adaptor (include/ghex_amd/field_descriptor.hpp) driven like a GHEX
communication_object would drive a field descriptor, checked against the oracle."""
import os
import subprocess

import numpy as np
import pytest

from oracle import oracle as orc
from tests import helpers as H

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "cpp", "bin", "adaptor_demo")


def test_adaptor_header_compiles_host_only(tmp_path):
    src = tmp_path / "t.cpp"
    src.write_text('#include <ghex_amd/field_descriptor.hpp>\n'
                   'int main(){ ghex_amd::structured::field_descriptor<double,3> f(0,nullptr,'
                   '{1,1,1},{4,4,4},{2,1,0}); return f.byte_strides()[2] == 128 ? 0 : 1; }\n')
    exe = tmp_path / "t"
    subprocess.run(["g++", "-std=c++17", "-I", os.path.join(ROOT, "include"), str(src), "-o",
                    str(exe), "-L", os.path.join(ROOT, "ghex_amd", "lib"), "-lghx",
                    f"-Wl,-rpath,{os.path.join(ROOT, 'ghex_amd', 'lib')}"], check=True)
    assert subprocess.run([str(exe)]).returncode == 0


def test_data_descriptor_header_compiles_host_only(tmp_path):
    src = tmp_path / "u.cpp"
    src.write_text('#include <ghex_amd/data_descriptor.hpp>\n'
                   'int main(){ ghex_amd::unstructured::data_descriptor<int,double> d(3,100,nullptr,'
                   '4,false); return (d.desc().level_stride == 100 && d.desc().index_stride == 1'
                   ' && d.num_components() == 4) ? 0 : 1; }\n')
    exe = tmp_path / "u"
    subprocess.run(["g++", "-std=c++17", "-I", os.path.join(ROOT, "include"), str(src), "-o",
                    str(exe), "-L", os.path.join(ROOT, "ghex_amd", "lib"), "-lghx",
                    f"-Wl,-rpath,{os.path.join(ROOT, 'ghex_amd', 'lib')}"], check=True)
    assert subprocess.run([str(exe)]).returncode == 0


@pytest.mark.gpu
@pytest.mark.parametrize("N,Hw", [(8, 2), (10, 3), (7, 1)])
def test_cpp_adaptor_self_exchange(tmp_path, N, Hw):
    assert os.path.exists(EXE), "build() compiles tests/cpp/bin/adaptor_demo"
    pre = str(tmp_path / "out")
    subprocess.run([EXE, str(N), str(Hw), pre], check=True, timeout=120)
    ranks, gf, gl = H.cube_domains(N, (1, 1, 1))
    a, spec = H.linear_index_field(ranks[0][0], N, Hw, gl)
    opat = orc.regular_make_pattern(ranks, gf, gl, (Hw,) * 6, (1, 1, 1))
    (key, ob), = orc.regular_exchange([[(spec, 0, 0, 0)]], {0: opat}, 1).items()
    buf = np.fromfile(pre + ".buf", dtype=np.uint8)
    field = np.fromfile(pre + ".field", dtype=np.float64).reshape(a.shape)
    np.testing.assert_array_equal(buf, ob)
    np.testing.assert_array_equal(field, a)


UEXE = os.path.join(ROOT, "tests", "cpp", "bin", "udata_demo")


@pytest.mark.gpu
@pytest.mark.parametrize("levels,levels_first,lid_bytes", [(1, True, 8), (3, True, 4),
                                                           (4, False, 8), (2, False, 4)])
def test_cpp_unstructured_adaptor(tmp_path, levels, levels_first, lid_bytes):
    """include/ghex_amd/data_descriptor.hpp: pack / unpack of one neighbour's index list vs the
    oracle's data_descriptor get/set (user_concepts.hpp:385-440)."""
    assert os.path.exists(UEXE), "build() compiles tests/cpp/bin/udata_demo"
    rng = np.random.default_rng(11)
    n = 5000
    lids = rng.choice(n, size=777, replace=False).astype(np.int64)
    lf = tmp_path / "lids.bin"
    lids.tofile(lf)
    pre = str(tmp_path / "out")
    subprocess.run([UEXE, str(n), str(levels), "1" if levels_first else "0", str(lid_bytes),
                    str(lf), pre], check=True, timeout=120)
    isd, lsd = (levels, 1) if levels_first else (1, n)
    vals = np.zeros(n * levels)
    for i in range(n):
        for l in range(levels):
            vals[i * isd + l * lsd] = i * 100 + l
    ob = np.zeros(len(lids) * levels * 8, np.uint8)
    orc.unstructured_get(vals, ob, 8, lids, levels, levels_first, isd, lsd)
    np.testing.assert_array_equal(np.fromfile(pre + ".buf", dtype=np.uint8), ob)
    rb = (1e6 + np.arange(len(lids) * levels)).astype(np.float64)
    exp = vals.copy()
    orc.unstructured_set(exp, rb.view(np.uint8), 8, lids, levels, levels_first, isd, lsd)
    np.testing.assert_array_equal(np.fromfile(pre + ".values", dtype=np.float64), exp)
    # the list reversed in place at the same address: a new plan, not the cached one
    ob2 = np.zeros(len(lids) * levels * 8, np.uint8)
    orc.unstructured_get(exp, ob2, 8, lids[::-1].copy(), levels, levels_first, isd, lsd)
    np.testing.assert_array_equal(np.fromfile(pre + ".buf2", dtype=np.uint8), ob2)
    # then entries 1 and 2 swapped in place, between the 16 sampled positions:
    # the exact check builds a new plan
    rl = lids[::-1].copy()
    rl[[1, 2]] = rl[[2, 1]]
    ob3 = np.zeros(len(lids) * levels * 8, np.uint8)
    orc.unstructured_get(exp, ob3, 8, rl, levels, levels_first, isd, lsd)
    np.testing.assert_array_equal(np.fromfile(pre + ".buf3", dtype=np.uint8), ob3)
    assert int(open(pre + ".plans").read()) == 2  # LRU bound held
