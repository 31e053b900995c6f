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
