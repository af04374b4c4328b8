"""Generate tests/golden/reference_kats.json from the reference's own tests.

Run in the build container (where /root/reference exists):
    python tools/make_golden_kats.py

The output is DATA only: the input vectors, graph snapshot and expected
answers that the reference's tests hold, each tagged with the file:line it
comes from.  No reference source text is copied.
"""
import json
import os
import re

REF = "/root/reference/adapters/repos/db/vector/hnsw"
OUT = os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "reference_kats.json")


def parse_vectors_for_delete_test():
    src = open(os.path.join(REF, "delete_test.go")).read()
    body = src[src.index("func vectorsForDeleteTest() [][]float32 {"):]
    body = body[: body.index("\n}\n")]
    rows = re.findall(r"\{([-0-9.e, ]+)\}", body)
    return [[float(x) for x in r.split(",")] for r in rows]


def parse_json_snapshot():
    src = open(os.path.join(REF, "delete_test.go")).read()
    start = src.index("func TestDelete_Flakyness_gh_1369")
    seg = src[start:]
    m = re.search(r"snapshotBefore := \[\]byte\(`(.*?)`\)", seg, re.S)
    return json.loads(m.group(1))


def main():
    kats = {
        "distancer": {
            "source": "distancer/l2_test.go:21-66, dot_product_test.go:21-66, cosine_dist_test.go:21-82",
            "l2": [
                {"a": [3, 4, 5], "b": [3, 4, 5], "expect": 0.0},
                {"a": [3, 4, 5], "b": [1.5, 2, 2.5], "expect": 12.5},
                {"a": [10, 11], "b": [13, 15], "expect": 25.0},
            ],
            "dot": [
                {"a": [3, 4, 5], "b": [3, 4, 5], "expect": -50.0},
                {"a": [0, 1, 0, 2, 0, 3], "b": [1, 0, 2, 0, 3, 0], "expect": 0.0},
                {"a": [3, 4, 5], "b": [-3, -4, -5], "expect": 50.0},
            ],
            # inputs are normalized first (Normalize), expectations with delta
            "cosine": [
                {"a": [0.1, 0.3, 0.7], "b": [0.1, 0.3, 0.7], "expect": 0.0, "delta": 0.0},
                {"a": [0.1, 0.3, 0.7], "b": [0.2, 0.6, 1.4], "expect": 0.0, "delta": 0.0},
                {"a": [0.1, 0.3, 0.7], "b": [0.2, 0.2, 0.2], "expect": 0.173, "delta": 0.01},
                {"a": [0.1, 0.3, 0.7], "b": [-0.1, -0.3, -0.7], "expect": 2.0, "delta": 0.01},
            ],
            "asm_vs_purego_lengths": {
                "source": "distancer/l2_amd64_test.go:35-73 (InEpsilon 0.01)",
                "lengths": [1, 4, 16, 31, 32, 35, 64, 67, 128, 130, 256, 260, 384, 390, 768, 777],
                "epsilon": 0.01,
            },
        },
        "acceptance_distances": {
            "source": "test/acceptance/vector_distances/{l2,dot,cosine}_test.go",
            "l2": {"objects": [[10, 11, 12], [13, 15, 17], [0, 0, 0]], "query": [10, 11, 12],
                   "expect": [0, 50, 365], "limited": {"distance": 364, "expect": [0, 50]}},
            "dot": {"objects": [[3, 4, 5], [1, 1, 1], [0, 0, 0], [-3, -4, -5]], "query": [3, 4, 5],
                    "expect": [-50, -12, 0, 50],
                    "limited": [{"distance": 30, "expect": [-50, -12, 0]},
                                {"distance": 0, "expect": [-50, -12, 0]},
                                {"distance": -40, "expect": [-50]},
                                {"distance": -60, "expect": []}]},
            "cosine": {"objects": [[0.7, 0.3], [1.4, 0.6], [-0.7, -0.3], [1, 1]], "query": [0.7, 0.3],
                       "expect": [0, 0, 0.0715, 2], "delta": 0.01},
        },
        "priority_queue": {
            "source": "priorityqueue/queue_test.go:20-82",
            "values": {"0": 0.0, "1": 0.23, "2": 0.8, "3": 0.222, "4": 0.88, "5": 1.0},
            "min_order": [0, 3, 1, 2, 4, 5],
            "max_order": [5, 4, 2, 1, 3, 0],
        },
        "dynamic_ef": {
            "source": "dynamic_ef_test.go:27-102",
            "cases": [
                {"ef": -1, "min": 100, "max": 500, "factor": 8, "k": 100, "expect": 500},
                {"ef": -1, "min": 100, "max": 500, "factor": 8, "k": 10, "expect": 100},
                {"ef": -1, "min": 100, "max": 500, "factor": 8, "k": 23, "expect": 184},
                {"ef": 78, "min": 0, "max": 0, "factor": 0, "k": 5, "expect": 78},
            ],
        },
        "search_by_dist_params": {
            "source": "search_by_dist_test.go:20-32",
            "iterations": [{"offset": 0, "limit": 100, "total": 100}, {"offset": 100, "limit": 1000, "total": 1100}],
        },
        "index_clusters": {
            "source": "index_test.go:24-63, vectors_for_test.go:17-29, index_test.go:126-144",
            "metric": "cosine-dot", "max_connections": 30, "ef_construction": 60,
            "vectors": [[0.1, 0.9], [0.15, 0.8], [0.13, 0.65], [0.6, 0.1], [0.63, 0.2], [0.65, 0.08],
                        [0.8, 0.8], [0.9, 0.75], [0.8, 0.7]],
            "queries": [
                {"position": 0, "k": 3, "ef": 36, "expect_set": [0, 1, 2]},
                {"position": 3, "k": 3, "ef": 36, "expect_set": [3, 4, 5]},
                {"position": 6, "k": 3, "ef": 36, "expect_set": [6, 7, 8]},
                {"position": 3, "k": 50, "ef": 36, "expect_order": [3, 5, 4, 7, 8, 6, 2, 1, 0]},
            ],
        },
        "hand_built_graph": {
            "source": "search_test.go:26-89",
            "metric": "l2-squared", "max_connections": 30, "ef_construction": 128,
            "vectors": [[100, 100], [2, 2], [1, 1]],
            "entrypoint": 0, "max_level": 1,
            "nodes": [{"id": 0, "level": 1, "connections": [[1, 2], [1]]},
                      {"id": 2, "level": 0, "connections": [[0, 1, 2]]}],
            "nil_nodes": [1],
            "query": [1.7, 1.7], "k": 20, "expect": [2, 0], "expect_tombstoned": [1],
        },
        "delete_snapshot": {
            "source": "delete_test.go:1092-1150 (snapshot), :712-760 (vectors), debug.go:143-175 (loader: cosine, M=30)",
            "metric": "cosine-dot", "max_connections": 30, "ef_construction": 128,
            "vectors": parse_vectors_for_delete_test(),
            "snapshot": parse_json_snapshot(),
            "query": [0.1, 0.1, 0.1], "k": 20,
            "allow": "odd ids", "tombstone_after": [30, 32, 34, 36],
            "invariant": "search(allow=odd) == search after tombstoning the listed even ids",
        },
        "allow_list_iteration": {
            "source": "helpers/allow_list_test.go:103-133",
            "insert": [3, 2, 1], "expect_iteration": [1, 2, 3],
        },
    }
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    with open(OUT, "w") as f:
        json.dump(kats, f, indent=1)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
