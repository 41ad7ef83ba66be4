"""Where the upload path sits on the box: the GPU's PCI device and NUMA node,
the CPUs this process may run on and their nodes, and a pinned host buffer's
pages by node (first-touched by this process, as the library's pinned upload
ring is) — the facts behind the one-shot / stream H2D rates.

usage: python tools/numa_probe.py   (prints one JSON line)
"""
import ctypes
import glob
import json
import os
import re


def cpu_nodes():
    nodes = {}
    for d in glob.glob("/sys/devices/system/node/node[0-9]*"):
        n = int(d.rsplit("node", 1)[1])
        for part in open(os.path.join(d, "cpulist")).read().strip().split(","):
            if not part:
                continue
            a, _, b = part.partition("-")
            for c in range(int(a), int(b or a) + 1):
                nodes[c] = n
    return nodes


def gpu_pci():
    hip = ctypes.CDLL("libamdhip64.so")
    buf = ctypes.create_string_buffer(64)
    if hip.hipDeviceGetPCIBusId(buf, 64, 0) != 0:
        return None, None
    bdf = buf.value.decode().lower()
    node = None
    for cand in (bdf, bdf[:-1] + "0"):
        p = "/sys/bus/pci/devices/%s/numa_node" % cand
        if os.path.exists(p):
            node = int(open(p).read().strip())
            break
    return bdf, node


def pinned_pages_by_node(nbytes=64 << 20):
    hip = ctypes.CDLL("libamdhip64.so")
    p = ctypes.c_void_p()
    if hip.hipHostMalloc(ctypes.byref(p), ctypes.c_size_t(nbytes), 0) != 0:
        return None
    ctypes.memset(p, 1, nbytes)
    lo, hi = p.value, p.value + nbytes
    counts = {}
    for line in open("/proc/self/numa_maps"):
        addr = int(line.split()[0], 16)
        if lo <= addr < hi or (addr <= lo < addr + nbytes):
            for m in re.finditer(r"\bN(\d+)=(\d+)", line):
                counts[int(m.group(1))] = counts.get(int(m.group(1)), 0) + int(m.group(2))
    hip.hipHostFree(p)
    return counts


def main():
    nodes = cpu_nodes()
    aff = sorted(os.sched_getaffinity(0))
    by_node = {}
    for c in aff:
        by_node.setdefault(nodes.get(c, -1), []).append(c)
    bdf, gnode = gpu_pci()
    out = {"gpu_pci": bdf, "gpu_numa_node": gnode, "numa_nodes": len(set(nodes.values())),
           "allowed_cpus": len(aff), "allowed_cpus_by_node": {str(k): len(v) for k, v in sorted(by_node.items())},
           "pinned_64MiB_pages_by_node": pinned_pages_by_node()}
    try:
        out["cgroup_cpu_max"] = open("/sys/fs/cgroup/cpu.max").read().strip()
    except OSError:
        pass
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
