"""Pin the oracle (oracle/) against the reference's own outputs and known-answer tests.

* regular halo boxes + intersections: tests/golden/ref_halo_boxes.json, produced by the
  reference's own halo_generator (halo_generator.hpp:93-160) compiled from /root/reference;
* unstructured pattern: the known-answer send/recv tables of
  test/unstructured/unstructured_test_case.hpp:217-343;
* full exchanges: the reference tests' self-validating properties
  (test_regular_domain.cpp:739-800, unstructured_test_case.hpp:345-388,
  test_unstructured_domain_descriptor.py check_field).
"""
import json
import os

import numpy as np
import pytest

from oracle import oracle as orc
from tests import helpers as H


@pytest.fixture(scope="module")
def ref_boxes(golden_dir):
    with open(os.path.join(golden_dir, "ref_halo_boxes.json")) as fh:
        return json.load(fh)["configs"]


def test_halo_boxes_match_reference(ref_boxes):
    assert len(ref_boxes) > 200
    for c in ref_boxes:
        D = c["D"]
        got = orc.regular_halo_boxes(c["gfirst"], c["glast"], c["halos"], c["periodic"],
                                     c["dom"][0], c["dom"][1])
        exp = c["boxes"]
        assert len(got) == len(exp), c
        for b, e in zip(got, exp):
            assert list(b.lf) + list(b.ll) + list(b.gf) + list(b.gl) == e


def test_intersections_match_reference(ref_boxes):
    for c in ref_boxes:
        boxes = orc.regular_halo_boxes(c["gfirst"], c["glast"], c["halos"], c["periodic"],
                                       c["dom"][0], c["dom"][1])
        got = []
        for bi, b in enumerate(boxes):
            for k, (f, l) in enumerate(c["others"]):
                x = orc.intersect(b.lf, b.gf, b.gl, f, l)
                if all(a <= z for a, z in zip(x.gf, x.gl)):
                    got.append([bi, k] + list(x.lf) + list(x.ll) + list(x.gf) + list(x.gl))
        assert got == c["isect"]


def _unstructured_case(golden_dir):
    with open(os.path.join(golden_dir, "unstructured_case.json")) as fh:
        return json.load(fh)


def test_unstructured_known_answer_maps(golden_dir):
    case = _unstructured_case(golden_dir)
    doms = [[orc.UnstructuredDomain(int(k), v["gids"], v["halo_lids"])]
            for k, v in sorted(case["domains"].items())]
    for r, (inner, outer) in sorted(case["inner_outer"].items()):
        d = doms[int(r)][0]
        assert [d.gids[l] for l in sorted(d.inner.values())] == inner
        assert d.outer_gids == outer
    pats = orc.unstructured_make_pattern(doms)
    for r in range(4):
        p = pats[r][0]
        sends = {str(did): lids for (_, _), (did, lids) in p["send"].items()}
        recvs = {str(did): lids for (_, _), (did, lids) in p["recv"].items()}
        assert sends == case["send_maps"][str(r)]
        assert recvs == case["recv_maps"][str(r)]


@pytest.mark.parametrize("levels", [1, 3])
@pytest.mark.parametrize("levels_first", [True, False])
def test_unstructured_exchange_values(golden_dir, levels, levels_first):
    """test_user_concepts.cpp data_descriptor exchange + check_exchanged_data (:345-388)."""
    case = _unstructured_case(golden_dir)
    doms = [[orc.UnstructuredDomain(int(k), v["gids"], v["halo_lids"])]
            for k, v in sorted(case["domains"].items())]
    pats = orc.unstructured_make_pattern(doms)
    fields = []
    for r in range(4):
        d = doms[r][0]
        f = np.full(d.size() * levels, -1.0)
        for gid, lid in d.inner.items():
            for l in range(levels):
                idx = lid * levels + l if levels_first else lid + l * d.size()
                f[idx] = d.id * 10000 + gid * 100 + l
        fields.append(f)
    ist = lambda d: levels if levels_first else 1
    lst = lambda d: 1 if levels_first else d.size()
    msgs = {}
    for r in range(4):
        d = doms[r][0]
        for (rank, tag), (did, lids) in pats[r][0]["send"].items():
            buf = np.zeros(len(lids) * levels * 8, np.uint8)
            orc.unstructured_get(fields[r], buf, 8, lids, levels, levels_first, ist(d), lst(d))
            msgs[(r, rank, tag)] = buf
    for r in range(4):
        d = doms[r][0]
        for (rank, tag), (did, lids) in pats[r][0]["recv"].items():
            buf = msgs[(rank, r, tag)]
            orc.unstructured_set(fields[r], buf, 8, lids, levels, levels_first, ist(d), lst(d))
    for r in range(4):
        d = doms[r][0]
        for (rank, tag), (did, lids) in pats[r][0]["recv"].items():
            for lid in lids:
                for l in range(levels):
                    idx = lid * levels + l if levels_first else lid + l * d.size()
                    assert fields[r][idx] == did * 10000 + d.gids[lid] * 100 + l


def test_unstructured_python_fixture_repeated_gids_and_self(golden_dir):
    """test_unstructured_domain_descriptor.py: repeated halo gids + exchange with itself."""
    fx = _unstructured_case(golden_dir)["python_fixture"]
    L = fx["levels"]
    doms = [[orc.UnstructuredDomain(int(k), v["all"], v["outer_lids"])]
            for k, v in sorted(fx["domains"].items())]
    gids = [[v["outer"]] for k, v in sorted(fx["domains"].items())]
    pats = orc.unstructured_make_pattern(doms, gids)
    fields = []
    for r in range(4):
        d = doms[r][0]
        f = np.full((d.size(), L), -1, dtype=np.int64)
        for gid, lid in d.inner.items():
            f[lid] = [r * 1000 + 10 * gid + l for l in range(L)]
        fields.append(f)
    msgs = {}
    for r in range(4):
        for (rank, tag), (did, lids) in pats[r][0]["send"].items():
            buf = np.zeros(len(lids) * L * 8, np.uint8)
            orc.unstructured_get(fields[r], buf, 8, lids, L, True, L, 1)
            msgs[(r, rank, tag)] = buf
    assert any(k[0] == k[1] for k in msgs), "fixture has a self-exchange"
    for r in range(4):
        for (rank, tag), (did, lids) in pats[r][0]["recv"].items():
            orc.unstructured_set(fields[r], msgs[(rank, r, tag)], 8, lids, L, True, L, 1)
    for r in range(4):
        d = doms[r][0]
        for lid, gid in enumerate(d.gids):
            for l in range(L):
                v = int(fields[r][lid, l])
                assert v % 1000 == 10 * gid + l, (r, lid, gid, v)


@pytest.mark.parametrize("types", [(np.float64, np.float32, np.int32),
                                   (np.float64, np.float64, np.float64)])
def test_structured_exchange_reference_geometry(types):
    """test_regular_domain.cpp run(): 6 fields (3 types x 2 domains), 2 patterns, one exchange."""
    ranks, gf, gl = H.regular_test_domains(4)
    pat1 = orc.regular_make_pattern(ranks, gf, gl, H.HALOS_1, (1, 1, 1))
    pat2 = orc.regular_make_pattern(ranks, gf, gl, H.HALOS_2, (1, 1, 1))
    patterns = {1: pat1, 2: pat2}
    arrays, ranks_fields = {}, []
    for r in range(4):
        flist = []
        for fi, (T, pc) in enumerate(zip(types, (1, 2, 1))):
            for li in range(2):
                dom = ranks[r][li]
                a = H.coord_field(dom, T)
                arrays[(r, fi, li)] = (a, dom, H.HALOS_1 if pc == 1 else H.HALOS_2)
                flist.append((H.coord_fieldspec(a), dom.id, li, pc))
        ranks_fields.append(flist)
    orc.regular_exchange(ranks_fields, patterns, 4)
    for (r, fi, li), (a, dom, halos) in arrays.items():
        assert H.check_coord_field(a, dom, halos, gf, gl) == 0, (r, fi, li)


@pytest.mark.parametrize("parts", [(1, 1, 1), (2, 1, 1), (2, 2, 2)])
@pytest.mark.parametrize("Hw", [1, 2, 3])
def test_structured_cube_exchange(parts, Hw):
    N = 8
    ranks, gf, gl = H.cube_domains(N, parts)
    pat = orc.regular_make_pattern(ranks, gf, gl, (Hw,) * 6, (1, 1, 1))
    fields = []
    rf = []
    for r, doms in enumerate(ranks):
        a, spec = H.linear_index_field(doms[0], N, Hw, gl)
        fields.append((a, doms[0]))
        rf.append([(spec, doms[0].id, 0, 0)])
    orc.regular_exchange(rf, {0: pat}, len(ranks))
    for a, dom in fields:
        np.testing.assert_array_equal(a, H.expected_linear_halo(a, dom, N, Hw, gl))


def test_cube_pattern_counts():
    """1-rank periodic = 1 key x 26 IS; 2x2x2 = 7 keys/rank (3 face peers x 2 IS,
    3 edge peers x 4 IS, 1 corner peer x 8 IS)."""
    ranks, gf, gl = H.cube_domains(8, (1, 1, 1))
    p = orc.regular_make_pattern(ranks, gf, gl, (2,) * 6, (1, 1, 1))[0][0]
    assert len(p.send) == 1 and len(list(p.send.values())[0][1]) == 26
    ranks, gf, gl = H.cube_domains(8, (2, 2, 2))
    p = orc.regular_make_pattern(ranks, gf, gl, (2,) * 6, (1, 1, 1))[5][0]
    sizes = sorted(len(v[1]) for v in p.send.values())
    assert sizes == [2, 2, 2, 4, 4, 4, 8]


def test_elementwise_equals_batch_for_unit_stride():
    N, Hw = 6, 2
    ranks, gf, gl = H.cube_domains(N, (1, 1, 1))
    p = orc.regular_make_pattern(ranks, gf, gl, (Hw,) * 6, (1, 1, 1))[0][0]
    lst = list(p.send.values())[0][1]
    for layout in [(2, 1, 0), (0, 1, 2), (1, 2, 0)]:
        a, spec = H.linear_index_field(ranks[0][0], N, Hw, gl, layout=layout)
        n = sum(b.size() for b in lst) * 8
        b1, b2 = np.zeros(n, np.uint8), np.zeros(n, np.uint8)
        assert orc.structured_pack(spec, b1, lst) == n
        orc.structured_pack(spec, b2, lst, elementwise=True)
        np.testing.assert_array_equal(b1, b2)


def _manifest():
    import json
    import os
    return json.load(open(os.path.join(os.path.dirname(__file__), "golden",
                                       "hash_manifest.json")))


def test_hash_manifest_small_cases_reproduce():
    """The committed checksum manifest (the GPU tests' expected values) is what the oracle
    produces today, for every small case (tests/golden/make_hash_manifest.py)."""
    from tests.golden.make_hash_manifest import case_name, run_case, small_cases
    m = _manifest()["small"]
    cases = list(small_cases())
    assert len(cases) == len(m) == 109
    for c in cases:
        assert run_case(*c) == m[case_name(*c)], case_name(*c)


def test_hash_manifest_full_sizes_and_message_counts():
    """Full-size entries: message sizes equal SURVEY §8(d)'s algorithmic bytes per direction
    (n(512,H) * 8 B on one rank; 2x2x2: 7 peer messages per rank, 3 faces of 2*N^2*H, 3 edges
    of 4*N*H^2, 1 corner of 8*H^3 elements)."""
    m = _manifest()["full"]
    n = {1: 1579016, 2: 3170368, 3: 4774104}
    for Hw, cells in n.items():
        e = m[f"N512_H{Hw}_L210_P111"]
        assert list(e["messages"].values())[0][0] == cells * 8
    e = m["N64_H2_L210_P222"]
    for r in range(8):
        sizes = sorted(v[0] for k, v in e["messages"].items() if k.startswith(f"{r}:"))
        N, Hw = 64, 2
        assert sizes == sorted([8 * 8 * Hw ** 3] + [8 * 4 * N * Hw * Hw] * 3
                               + [8 * 2 * N * N * Hw] * 3)
