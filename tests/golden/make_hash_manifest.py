"""Generate tests/golden/hash_manifest.json: FNV-1a-64 checksums of every packed message and of
every field after unpack, computed by the oracle (oracle/oracle.py regular_exchange, the
restatement of communication_object::pack/unpack + serialization<cpu>, pinned to the
reference's halo generator by tests/test_oracle.py). SURVEY.md §8(c) fixture plan, item 2.

Run in the build container:  python tests/golden/make_hash_manifest.py [--no-full]

Cases (all periodic, cube_domains geometry, owned cell = global linear index, halos -1):
  small: N in {8, 13} x H in {1, 2, 3} x the 6 layout maps x decompositions 1, (2,1,1), (2,2,2)
  asym : N=8, field offset 2, halos {0,0,1,0,1,2} (test_regular_domain.cpp pattern 1), (2,1,1)
  full : 512^3 fp64 H in {1, 2, 3} on one rank (BASELINE config 2), 2x2x2 at N=64 H=2, and
         2x2x2 ranks of 512^3 H=2 (BASELINE config 3 at full size; ~15 GB of host memory)
  config4: BASELINE config 4 (five mixed f64/f32 fields, H=3, 2x2x2) at N=7 and at full 256^3
  --only NAME updates one full / config4 case in the existing manifest.
The GPU tests recompute the same checksums from the HIP path (tests/test_gpu_manifest.py);
tests/test_oracle.py re-derives the small cases from the oracle (regression pin)."""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import oracle as orc  # noqa: E402
from tests import helpers as H  # noqa: E402

LAYOUTS = [(2, 1, 0), (0, 1, 2), (1, 2, 0), (2, 0, 1), (1, 0, 2), (0, 2, 1)]
PARTS = [(1, 1, 1), (2, 1, 1), (2, 2, 2)]
ASYM = (0, 0, 1, 0, 1, 2)


def case_name(N, Hw, layout, parts, halos=None):
    s = f"N{N}_H{Hw}_L{''.join(map(str, layout))}_P{''.join(map(str, parts))}"
    return s if halos is None else s + "_A" + "".join(map(str, halos))


def run_case(N, Hw, layout, parts, halos=None):
    """Oracle exchange of one linear-index field per rank. Returns the manifest entry:
    {"messages": {"<rank>:<recv dom>,<send dom>": [size, fnv]}, "fields": [fnv per rank]}."""
    halos = tuple(halos) if halos is not None else (Hw,) * 6
    ranks, gf, gl = H.cube_domains(N, parts)
    nr = len(ranks)
    opat = orc.regular_make_pattern(ranks, gf, gl, halos, (1, 1, 1))
    arrs, rf = [], []
    for r in range(nr):
        a, spec = H.linear_index_field(ranks[r][0], N, Hw, gl, layout=layout)
        arrs.append(a)
        rf.append([(spec, ranks[r][0].id, 0, 0)])
    bufs = orc.regular_exchange(rf, {0: opat}, nr)
    msgs = {f"{r}:{pair[0]},{pair[1]}": [int(b.size), f"{orc.fnv1a64(b):016x}"]
            for (r, pair), b in sorted(bufs.items())}
    return {"messages": msgs, "fields": [f"{orc.fnv1a64(a):016x}" for a in arrs]}


C4_TYPES = [np.float64, np.float32, np.float64, np.float32, np.float64]


def run_case_c4(N, Hw, parts):
    """BASELINE config 4: five fields [f64, f32, f64, f32, f64] per rank in ONE exchange (one
    message per domain pair, fields at alignof-padded offsets; pad bytes stay zero), owned cell =
    global linear index + field number (rounded to f32 where the field is f32), halos -1."""
    ranks, gf, gl = H.cube_domains(N, parts)
    nr = len(ranks)
    opat = orc.regular_make_pattern(ranks, gf, gl, (Hw,) * 6, (1, 1, 1))
    arrs, rf = [], []
    for r in range(nr):
        fl = []
        for k, T in enumerate(C4_TYPES):
            a, spec = H.linear_index_field(ranks[r][0], N, Hw, gl, dtype=T, add=k)
            arrs.append(a)
            fl.append((spec, ranks[r][0].id, 0, 0))
        rf.append(fl)
    bufs = orc.regular_exchange(rf, {0: opat}, nr)
    msgs = {f"{r}:{pair[0]},{pair[1]}": [int(b.size), f"{orc.fnv1a64(b):016x}"]
            for (r, pair), b in sorted(bufs.items())}
    return {"messages": msgs, "fields": [f"{orc.fnv1a64(a):016x}" for a in arrs]}


def c4_cases():
    yield (7, 3, (2, 2, 2))
    yield (256, 3, (2, 2, 2))


def c4_name(N, Hw, parts):
    return f"C4_N{N}_H{Hw}_P{''.join(map(str, parts))}"


def small_cases():
    for N in (8, 13):
        for Hw in (1, 2, 3):
            for layout in LAYOUTS:
                for parts in PARTS:
                    yield (N, Hw, layout, parts, None)
    yield (8, 2, (2, 1, 0), (2, 1, 1), ASYM)


def full_cases():
    for Hw in (1, 2, 3):
        yield (512, Hw, (2, 1, 0), (1, 1, 1), None)
    yield (64, 2, (2, 1, 0), (2, 2, 2), None)
    yield (512, 2, (2, 1, 0), (2, 2, 2), None)


def main(full=True):
    out = {"generator": "tests/golden/make_hash_manifest.py (oracle regular_exchange)",
           "hash": "FNV-1a 64 over the bytes (offset basis 0xcbf29ce484222325)",
           "small": {}, "full": {}}
    for c in small_cases():
        out["small"][case_name(*c)] = run_case(*c)
    if full:
        for c in full_cases():
            out["full"][case_name(*c)] = run_case(*c)
            print("full case", case_name(*c), flush=True)
        out["config4"] = {c4_name(*c): run_case_c4(*c) for c in c4_cases()}
    with open(os.path.join(HERE, "hash_manifest.json"), "w") as fh:
        json.dump(out, fh, indent=0, sort_keys=True)


def update_one(name):
    path = os.path.join(HERE, "hash_manifest.json")
    out = json.load(open(path))
    if name.startswith("C4_"):
        case = next(c for c in c4_cases() if c4_name(*c) == name)
        out.setdefault("config4", {})[name] = run_case_c4(*case)
    else:
        case = next(c for c in full_cases() if case_name(*c) == name)
        out["full"][name] = run_case(*case)
    with open(path, "w") as fh:
        json.dump(out, fh, indent=0, sort_keys=True)
    print("updated", name)


if __name__ == "__main__":
    if "--only" in sys.argv:
        update_one(sys.argv[sys.argv.index("--only") + 1])
    else:
        main(full="--no-full" not in sys.argv)
