"""What the box exposes without touching HIP (tools only): KFD topology nodes
(GPU or CPU, render minor, whether its render node is usable here), the
visibility env vars, the cgroup CPU quota and /dev/shm capacity."""
import glob
import json
import os

nodes = []
for p in sorted(glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties")):
    kv = {}
    try:
        for line in open(p):
            k, _, v = line.strip().partition(" ")
            kv[k] = v
    except OSError as e:
        kv = {"error": str(e)}
    minor = kv.get("drm_render_minor")
    dri = f"/dev/dri/renderD{minor}" if minor and minor != "0" else None
    nodes.append({"node": p.split("/")[-2], "gfx_target_version": kv.get("gfx_target_version"),
                  "drm_render_minor": minor, "location_id": kv.get("location_id"), "domain": kv.get("domain"),
                  "unique_id": kv.get("unique_id"), "render_exists": bool(dri and os.path.exists(dri)),
                  "render_rw": bool(dri and os.access(dri, os.R_OK | os.W_OK))})
env = {k: os.environ.get(k) for k in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES",
                                      "GPU_DEVICE_ORDINAL", "OMP_NUM_THREADS")}
try:
    quota = open("/sys/fs/cgroup/cpu.max").read().strip()
except OSError:
    quota = None
st = os.statvfs("/dev/shm")
print(json.dumps({"kfd_nodes": nodes, "env": env, "cpu.max": quota, "nproc": os.cpu_count(),
                  "affinity": len(os.sched_getaffinity(0)), "dev_dri": sorted(os.listdir("/dev/dri"))
                  if os.path.isdir("/dev/dri") else None, "kfd_rw": os.access("/dev/kfd", os.R_OK | os.W_OK),
                  "shm_free_GiB": round(st.f_bavail * st.f_frsize / 2**30, 1),
                  "mem_avail_GiB": round(int(next(l.split()[1] for l in open("/proc/meminfo")
                                                  if l.startswith("MemAvailable"))) / 2**20, 1)}))
