"""bench.py — decoded GB/s of the MI355X Parquet decoder (BASELINE.json metric).

Workload (BASELINE.json configs[1], the single-GPU headline config): one
required INT32 column, 100M rows, RLE_DICTIONARY pages whose index bit width
sweeps 1..20 across row groups (row group i uses a dictionary of 2^(1 + i % 20)
entries), Snappy, data page V1, ~1M-row row groups, 20k-row pages.  Synthetic
data (seeded), written with pyarrow on the box, then planned on the host and
uploaded to HBM once; the timed region is the whole GPU decode pipeline
(snappy -> prepare -> scan -> decode) with every page already resident.

`--config c1|c3|c4|c5` runs the other BASELINE.json configs through the same
pipeline (analysis lines; tools/synth.py describes their files).

A "step" decodes every page of the rank's shard once.  For N > 1 the file holds
N x 100M rows and each rank decodes a contiguous, byte-balanced slice of its
row groups (pqgpu.plan_row_group_shards) on its own GPU: weak scaling, no
collective on the data path; value = decoded bytes of all ranks / max-over-ranks
time.

Prints ONE JSON line (rank 0).
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "parquet-go_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import synth  # noqa: E402  (tools/synth.py: the configs' synthetic files)

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def cpu_baseline(path, budget_s=10.0, threads=None, min_s=1.0):
    """The CPU oracle (a C port of the reference read path) on a bounded sample
    of the same file: whole row groups, one per worker thread at a time (the
    oracle releases the GIL inside its C calls), until ~budget_s of wall time.
    `threads` defaults to the 16-core CPU share of a GPU box."""
    import concurrent.futures as cf
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    data = open(path, "rb").read()
    f = oracle.File(data)
    L = oracle.lib()
    threads = threads or min(16, os.cpu_count() or 1)

    leaves = range(len(f.leaves()))

    def one(rg):
        # every selected leaf of the row group; output bytes as the GPU counts
        # them (values + validity + list offsets/validity + string offsets)
        nbytes, rows = 0, f.rg_num_rows(rg)
        for leaf in leaves:
            r = ctypes.c_void_p()
            st = L.pqref_decode(f._h, leaf, rg, rg + 1, ctypes.byref(r))
            if st != 0:
                raise RuntimeError("oracle failed on the bench file: %d" % st)
            for bid in (oracle.BUF_VALUES, oracle.BUF_VALIDITY, oracle.BUF_LIST_OFFSETS,
                        oracle.BUF_LIST_VALIDITY, oracle.BUF_STR_OFFSETS):
                n = ctypes.c_size_t()
                L.pqref_result_buffer(r, bid, ctypes.byref(n))
                nbytes += n.value
            L.pqref_result_free(r)
        return nbytes, rows

    out_bytes, rows, rgs = 0, 0, 0
    t0 = time.perf_counter()
    with cf.ThreadPoolExecutor(threads) as ex:
        rg = 0
        # whole passes over the file until ~min_s of wall (>= min_s x threads
        # CPU-seconds), stopping early at budget_s
        while time.perf_counter() - t0 < budget_s and (rg < f.num_row_groups or time.perf_counter() - t0 < min_s):
            wave = [(rg + k) % f.num_row_groups for k in range(min(threads, f.num_row_groups))]
            for nb, nr in ex.map(one, wave):
                out_bytes += nb
                rows += nr
            rgs += len(wave)
            rg += len(wave)
    t_total = time.perf_counter() - t0
    return {"value": out_bytes / t_total / 1e9, "unit": "GB/s", "cores": threads, "kind": "port",
            "sample": "oracle/pqref.c on %d threads, %d row-group decodes over the file's %d row groups (%d rows), %.1f s wall"
                      % (threads, rgs, f.num_row_groups, rows, t_total)}


def pmc_traffic(args, kernels=("k_expand", "k_decode", "k_dba")):
    """HBM bytes per launch of the decode phase from rocprofv3 PMC counters,
    collected in separate passes (FETCH_SIZE, then WRITE_SIZE) over a short
    child run of this same bench; MI355X_MICROARCH.md: on gfx950 FETCH_SIZE
    reports half of a wide streaming read, so it is doubled.  None when the
    profiler is unavailable or a pass fails."""
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile
    if not shutil.which("rocprofv3"):
        return None
    base = [sys.executable, os.path.abspath(__file__), "--no-cpu", "--no-pmc", "--steps", "3", "--warmup", "1",
            "--config", args.config, "--rows", str(args.rows), "--rg-rows", str(args.rg_rows), "--bw", str(args.bw)]
    if args.file:
        base += ["--file", args.file]
    per = {}
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as td:
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            out = os.path.join(td, ctr)
            cmd = ["timeout", "-s", "KILL", "120", "rocprofv3", "--pmc", ctr, "--output-format", "csv",
                   "-d", out, "-o", "run", "--"] + base
            try:
                subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, check=True, timeout=150)
            except Exception:
                return None
            vals = {}
            for f in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
                for r in csv.DictReader(open(f)):
                    if any(k in r["Kernel_Name"] for k in kernels) and r["Counter_Name"] == ctr:
                        vals.setdefault(r["Dispatch_Id"], 0.0)
                        vals[r["Dispatch_Id"]] += float(r["Counter_Value"])
            if not vals:
                return None
            per[ctr] = sorted(vals.values())
    # kilobytes per dispatch; one launch of the phase may be several dispatches (k_expand<4>, <8>, k_decode)
    n_launch = 4  # 1 warmup + 3 timed steps of the child run
    fetch = sum(per["FETCH_SIZE"]) / n_launch * 1024 * 2
    write = sum(per["WRITE_SIZE"]) / n_launch * 1024
    return fetch + write


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=sorted(synth.DEFAULTS))
    ap.add_argument("--rows", type=int, default=0, help="rows per GPU (default: the config's)")
    ap.add_argument("--rg-rows", type=int, default=0, help="rows per row group (default: the config's)")
    ap.add_argument("--file", default=None)
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 PMC passes behind roofline.traffic")
    ap.add_argument("--bw", type=int, default=0, help="analysis: one dictionary bit width for every row group")
    args = ap.parse_args()
    args.rows = args.rows or synth.DEFAULTS[args.config][0]
    args.rg_rows = args.rg_rows or synth.DEFAULTS[args.config][1]

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")

    def barrier():
        if dist is not None:
            dist.barrier()

    import pqgpu
    total_rows = args.rows * world
    path = args.file or os.path.join(os.environ.get("TMPDIR", "/tmp"),
                                     "pqgpu_bench_%s_%d_%d_%d.parquet" % (args.config, total_rows, args.rg_rows, args.bw))
    if local == 0 and not os.path.exists(path):
        synth.make(args.config, path, total_rows, args.rg_rows, fixed_bw=args.bw)
    barrier()

    ctx = pqgpu.Context(local if world > 1 else 0)
    reader = pqgpu.FileReader(path, ctx=ctx)
    sizes = [reader.RowGroupByteSize(i) for i in range(reader.RowGroupCount())]
    rg0, rg1 = pqgpu.plan_row_group_shards(sizes, world)[rank]
    reader.batch(rg0, rg1).close()  # first use: HIP runtime and pinned ring set-up
    t_create = time.perf_counter()
    batch = reader.batch(rg0, rg1)  # host plan (page headers) + one H2D upload of the chunks
    t_create = time.perf_counter() - t_create
    stats = batch.stats()

    def step():
        batch.decode()

    for _ in range(args.warmup):
        step()
    batch.sync()
    batch.kernel_times()  # drop warmup events
    # the decode phase is bracketed by HIP events on a sample of the timed steps
    # (each event pair costs a few us of launch gap); at least 5 samples
    batch.set_timing(max(1, args.steps // 5))
    barrier()
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipDeviceSynchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    hip.hipDeviceSynchronize()
    barrier()
    dt = time.perf_counter() - t0
    batch.sync()  # raises if any page failed to decode
    # per-kernel HIP-event times recorded on the decode stream during the timed steps
    kern = {k: [v] for k, v in batch.kernel_times().items()}
    out_b, in_b = stats["output_bytes"], stats["input_bytes"]
    job_out = out_b
    if dist is not None:
        import torch
        t = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)  # the slowest rank sets the job time
        dt = float(t.item())
        nb = torch.tensor([out_b], dtype=torch.float64, device="cuda")
        dist.all_reduce(nb, op=dist.ReduceOp.SUM)  # every rank's decoded bytes
        job_out = float(nb.item())

    per_step = dt / args.steps
    value = job_out * args.steps / dt / 1e9
    avg = {k: float(np.mean(v)) for k, v in kern.items()}
    dom = max(avg, key=avg.get)
    # algorithmic bytes per launch of each kernel
    alg = {
        "k_snappy+k_copy": stats["input_bytes"] + stats["staged_bytes"],     # compressed in + uncompressed out
        "k_decode+k_expand": in_b + out_b,                                         # encoded pages in + decoded values out
    }
    ach = alg.get(dom, in_b + out_b) / (avg[dom] * 1e-3) / 1e9
    line = {
        "metric": "decoded GB/s (uncompressed output) per GPU + node at 1/2/4/8 MI355X, % HBM peak",
        "value": round(value, 3),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(per_step * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": synth.DTYPE[args.config],
        "data": "synthetic (seeded pyarrow writer on the box, tools/synth.py %s)" % args.config,
        "config": {"workload": synth.DESCR[args.config] % (args.rows, args.rg_rows),
                   "rows_per_gpu": args.rows, "row_groups": [rg0, rg1],
                   "pages": stats["data_pages"], "dict_pages": stats["dict_pages"],
                   "B_in": in_b, "B_out": out_b, "staged": stats["staged_bytes"],
                   "pipeline_hbm_frac": round((in_b + out_b) / per_step / 1e9 / HBM_PEAK_GBPS, 4),
                   "kernel_ms": {k: round(v, 4) for k, v in avg.items()},
                   # PCIe-inclusive rate (not `value`): host planning + H2D upload + one step
                   "e2e": {"batch_create_ms": round(t_create * 1e3, 2),
                           "GBps_incl_plan_and_h2d": round(out_b / (t_create + per_step) / 1e9, 1)},
                   "parallelism": "row-group shards, one process per GPU, no data-path collective"},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(ach, 1), "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBPS, 4), "traffic": None},
    }
    if rank == 0 and not args.no_cpu:
        line["cpu_baseline"] = cpu_baseline(path, args.cpu_budget)
    if rank == 0 and world == 1 and not args.no_pmc:
        tr = pmc_traffic(args)
        line["roofline"]["traffic"] = None if tr is None else round(tr / 1e6, 1)
        line["roofline"]["traffic_unit"] = "MB per launch (FETCH_SIZE x 2 + WRITE_SIZE)"
    if rank == 0:
        print(json.dumps(line), flush=True)
    batch.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
