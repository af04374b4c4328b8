"""Hash of the sources that define the f16 key pass (kernel + its launch), so a
PMC summary in profiles/ is attached to a bench line only when it was collected
from the same code (bench.py attach_traffic; tools/pmc_h16.sh writes it)."""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SOURCES = ("wv_h16.hip", "wv_h16_dev.h", "wv_topk.h", "wv_api.hip", "wv_params.h", "wv_device.h")
# the HNSW search kernel and its launch
SOURCES_HNSW = ("wv_hnsw.hip", "wv_api.hip", "wv_params.h", "wv_device.h")


def build_hash(kernel: str = "wv_bf_h16_kernel") -> str:
    h = hashlib.sha1()
    for name in (SOURCES_HNSW if "hnsw" in kernel else SOURCES):
        with open(os.path.join(ROOT, "weaviate_amd", "csrc", name), "rb") as f:
            h.update(name.encode() + b"\0" + f.read())
    return h.hexdigest()[:16]


def host_cores_info() -> dict:
    """CPUs this process may use: the affinity mask, capped by a cgroup CPU
    quota (v2 cpu.max or v1 cfs_quota) and by the OMP_NUM_THREADS share the
    GPU box sets (it shares a big host: os.cpu_count() shows every CPU)."""
    info = {"affinity": len(os.sched_getaffinity(0))}
    for path in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        try:
            with open(path) as f:
                parts = f.read().split()
            if path.endswith("cpu.max") and parts[0] != "max":
                info["cgroup_quota"] = max(1, int(parts[0]) // int(parts[1]))
            elif path.endswith("quota_us") and int(parts[0]) > 0:
                with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                    info["cgroup_quota"] = max(1, int(parts[0]) // int(f.read()))
        except (OSError, ValueError, IndexError):
            pass
    if os.environ.get("OMP_NUM_THREADS", "").isdigit():
        info["omp_num_threads"] = int(os.environ["OMP_NUM_THREADS"])
    info["cores"] = min(v for v in info.values())
    return info


def host_cores() -> int:
    return host_cores_info()["cores"]


if __name__ == "__main__":
    print(host_cores() if sys.argv[1:] == ["cores"] else build_hash())
