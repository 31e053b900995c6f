"""Generate tests/golden/unstructured_case.json (run in the build container; needs /root/reference).

Holds the reference's own known-answer unstructured test data:
  * test/unstructured/unstructured_test_case.hpp:35-86  (4 domains: gids + halo lids),
    :217-279 (send maps), :281-343 (recv maps), :345-388 (value encoding) — transcribed below;
  * test/bindings/python/test_unstructured_domain_descriptor.py:45-213 (4 domains with repeated
    halo gids and self-exchange) — the `domains = {...}` literal is read from the file as data.
"""
import ast
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
REF_PY = "/root/reference/test/bindings/python/test_unstructured_domain_descriptor.py"

case = {
    "source": "test/unstructured/unstructured_test_case.hpp:35-388",
    "domains": {
        "0": {"gids": [0, 13, 5, 2, 1, 3, 7, 11, 20], "halo_lids": [4, 5, 6, 7, 8]},
        "1": {"gids": [1, 19, 20, 4, 7, 15, 8, 0, 9, 13, 16], "halo_lids": [7, 8, 9, 10]},
        "2": {"gids": [3, 16, 18, 1, 5, 6], "halo_lids": [3, 4, 5]},
        "3": {"gids": [17, 6, 11, 10, 12, 9, 0, 3, 4], "halo_lids": [6, 7, 8]}},
    "inner_outer": {"0": [[0, 13, 5, 2], [1, 3, 7, 11, 20]],
                    "1": [[1, 19, 20, 4, 7, 15, 8], [0, 9, 13, 16]],
                    "2": [[3, 16, 18], [1, 5, 6]], "3": [[17, 6, 11, 10, 12, 9], [0, 3, 4]]},
    # send_maps[sender][receiver] = local indices on the send side
    "send_maps": {"0": {"1": [0, 1], "2": [2], "3": [0]}, "1": {"0": [0, 4, 2], "2": [0], "3": [3]},
                  "2": {"0": [0], "1": [1], "3": [0]}, "3": {"0": [2], "1": [5], "2": [1]}},
    # recv_maps[receiver][sender] = local indices on the recv side
    "recv_maps": {"0": {"1": [4, 6, 8], "2": [5], "3": [7]},
                  "1": {"0": [7, 9], "2": [10], "3": [8]},
                  "2": {"0": [4], "1": [3], "3": [5]}, "3": {"0": [6], "1": [8], "2": [7]}},
    "value_encoding": "dom*10000 + gid*100 + level",
}

if __name__ == "__main__":
    src = open(REF_PY).read()
    body = src[src.index("domains = {"):src.index("# fmt: on")]
    # the text after "domains = " is a dict literal of integers: parsed as data, never executed
    literal = body[body.index("{"):].strip()
    domains = ast.literal_eval(literal)
    py = {str(k): {kk: v[kk] for kk in ("all", "outer", "outer_lids", "inner")}
          for k, v in domains.items()}
    case["python_fixture"] = {
        "source": "test/bindings/python/test_unstructured_domain_descriptor.py:45-213, LEVELS=2",
        "levels": 2, "value_encoding": "rank*1000 + 10*gid + level", "domains": py}
    with open(os.path.join(HERE, "unstructured_case.json"), "w") as fh:
        json.dump(case, fh, indent=1)
