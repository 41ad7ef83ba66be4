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
N x 100M rows and each rank decodes a contiguous slice of its row groups,
balanced by estimated decode cost (pqgpu.plan_row_group_shards over
FileReader.RowGroupCost) on its own GPU: weak scaling, no
collective on the data path; value = decoded bytes of all ranks / max-over-ranks
time.  `--gpus N` without WORLD_SIZE in the environment starts the N rank
processes itself (spawn_ranks); under torch.distributed.run WORLD_SIZE must
equal N.  `--allgather` additionally times the optional column all-gather and the
all-to-one gather to rank 0 over RCCL (pqgather, never inside the timed steps).

Besides the timed loop (rank 0, N = 1), outside the timed region:
  * every pipeline phase is timed with HIP events on a second batch of the
    same shard (PQG_SEGMENT_TIMES=1); the longest phase is `roofline`'s, with
    its own algorithmic bytes;
  * a `rocprofv3 --kernel-trace --stats` child run gives per-kernel durations
    and calls of its last CHILD_STEPS decode steps (`roofline.kernel` = the
    longest kernel of that phase, `frac_from_trace` = the phase's bytes over
    its kernels' traced time per step) and two `--pmc` child runs give
    FETCH_SIZE / WRITE_SIZE per kernel per step (`roofline.traffic`: every
    dispatch of the phase's kernels in a step);
  * on every rank, the timed batch's own buffers (the whole shard, every
    leaf) are compared bit-exactly with the oracle's decode of the shard, and
    every row group is decoded again in a batch of its own and compared too
    (N > 1: a mismatch flag is all-reduced);
  * the CPU oracle (and pyarrow, when importable) decodes a bounded sample of
    the same file (cpu_baseline).

Prints ONE JSON line (rank 0).
"""
import argparse
import ctypes
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "parquet-go_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import synth  # noqa: E402  (tools/synth.py: the configs' synthetic files)

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec

# pipeline phases (pqg_batch_kernel_times names with PQG_SEGMENT_TIMES=1) and
# the kernels each one launches
PHASE_KERNELS = {
    "k_snappy+k_copy": ("k_snappy", "k_copy"),
    "k_dict_prepare": ("k_dict_prepare",),
    "k_prepare": ("k_prepare",),
    "k_scan": ("k_scan",),
    "k_decode+k_expand": ("k_decode", "k_expand", "k_dba"),
    "k_level_check": ("k_level_check",),
}


def phase_bytes(phase, st):
    """Algorithmic HBM bytes of one launch of a phase:
    snappy: compressed in + uncompressed out; dictionary prepare: dictionary
    pages in + 8-byte entries out (bounded by the page bytes); prepare: the
    data pages' stored bytes it walks; decode: encoded pages in + B_out."""
    return {
        "k_snappy+k_copy": st["snappy_in_bytes"] + st["staged_bytes"],
        "k_dict_prepare": 2 * st["dict_bytes"],
        "k_prepare": st["input_bytes"],
        "k_scan": 24 * st["pages"],
        "k_decode+k_expand": st["input_bytes"] + st["output_bytes"],
        "k_level_check": 0,
    }[phase]


def cpu_cores():
    """Cores this process may use: the affinity set, capped by a cgroup CPU
    quota when one is set (the GPU box gives each GPU a share of the host)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(p)))
    except Exception:
        pass
    return (min(n, quota) if quota else n), n, quota


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except Exception:
        pass
    return platform.processor() or "unknown"


def cpu_decode_rate(path, threads, budget_s, min_s=1.0):
    """The CPU oracle (a C port of the reference read path) on whole row
    groups of the same file, one per worker thread at a time (the oracle
    releases the GIL inside its C calls), until ~budget_s of wall time."""
    import concurrent.futures as cf
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    data = open(path, "rb").read()
    f = oracle.File(data)
    L = oracle.lib()
    leaves = range(len(f.leaves()))

    def one(rg):
        # every leaf of the row group; output bytes as the GPU counts them
        # (values + validity + list offsets/validity + string offsets)
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
        while time.perf_counter() - t0 < budget_s and (rg < f.num_row_groups or time.perf_counter() - t0 < min_s):
            wave = [(rg + k) % f.num_row_groups for k in range(min(threads, f.num_row_groups))]
            for nb, nr in ex.map(one, wave):
                out_bytes += nb
                rows += nr
            rgs += len(wave)
            rg += len(wave)
    dt = time.perf_counter() - t0
    return out_bytes / dt / 1e9, rgs, rows, dt, f.num_row_groups


def cpu_baseline(path, budget_s=8.0):
    """CPU oracle on all usable host cores and on one core (SURVEY.md §8(d):
    T = all host cores, plus the single-thread figure; the Go reference
    itself cannot run here — no Go toolchain)."""
    cores, affinity, quota = cpu_cores()
    v, rgs, rows, dt, nrg = cpu_decode_rate(path, cores, budget_s)
    v1, rgs1, rows1, dt1, _ = cpu_decode_rate(path, 1, budget_s / 2)
    return {"value": round(v, 3), "unit": "GB/s", "cores": cores, "kind": "port",
            "value_1_thread": round(v1, 3),
            "cpu_model": cpu_model(), "nproc": os.cpu_count(), "affinity_cpus": affinity, "cgroup_cpu_quota": quota,
            "sample": "oracle/pqref.c (C port of the reference read path): %d threads, %d row-group decodes over "
                      "the file's %d row groups (%d rows), %.1f s wall; 1 thread: %d row groups, %.1f s"
                      % (cores, rgs, nrg, rows, dt, rgs1, dt1)}


def _kname(s):
    """'void pq::k_decode<2>(pq::KArgs)' -> 'k_decode<2>'"""
    return s.split("(")[0].replace("void ", "").replace("pq::", "").strip()


def _child_cmd(args, steps=3):
    cmd = [sys.executable, os.path.abspath(__file__), "--child", "--steps", str(steps), "--warmup", "1",
           "--config", args.config, "--rows", str(args.rows), "--rg-rows", str(args.rg_rows), "--bw", str(args.bw)]
    if args.file:
        cmd += ["--file", args.file]
    return cmd


# every full decode ends with the same launch (pq_host.cpp launch_all):
# k_level_check, or — in a batch without level streams, which skips it — the
# last tiled-expand launch; the child's timed loop is the last thing it
# launches, so the dispatches after the (CHILD_STEPS + 1)-th last step end are
# exactly CHILD_STEPS decode steps
CHILD_STEPS = 3
STEP_END = "k_level_check"


def _step_end(rows, key_name):
    """The kernel that ends every decode of this run: k_level_check when it is
    launched, else the run's last dispatch of a pq kernel (host submission
    order)."""
    if any(_kname(r[key_name]) == STEP_END for r in rows):
        return STEP_END
    ours = [r for r in rows if not r[key_name].startswith("__amd")]  # (the runtime's blit kernels: copies)
    return _kname(ours[-1][key_name]) if ours else STEP_END


def _last_steps(rows, key_id, key_name, steps=CHILD_STEPS):
    """Rows of the last `steps` decode steps, in dispatch (host submission) order."""
    rows = sorted(rows, key=lambda r: int(r[key_id]))
    end = _step_end(rows, key_name)
    ends = [i for i, r in enumerate(rows) if _kname(r[key_name]) == end]
    if len(ends) < steps + 1:
        return None
    # every step launches the same sequence: if the end kernel ran more than
    # once a step, the segments between its dispatches would differ — refuse
    # the per-step split rather than cut the trace into wrong steps
    segs = [[_kname(r[key_name]) for r in rows[ends[-k - 1] + 1:ends[-k] + 1] if not r[key_name].startswith("__amd")]
            for k in range(1, steps + 1)]
    if any(sg != segs[0] for sg in segs[1:]):
        return None
    return rows[ends[-steps - 1] + 1:ends[-1] + 1]


def kernel_trace(args):
    """Per-kernel figures of the timed steps of a rocprofv3 --kernel-trace
    --stats child run of this same bench: {kernel: {avg_us, calls_per_step,
    us_per_step}} over the child's last CHILD_STEPS decode steps (None if
    rocprofv3 is unavailable).  With PQG_BENCH_PROF_DIR the run's own
    kernel_stats.csv, its per-dispatch kernel_trace.csv and the per-step
    summary (rocprof_kernel_steps_<cfg>.csv) are kept there."""
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile
    if not shutil.which("rocprofv3"):
        return None
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as td:
        cmd = ["timeout", "-s", "KILL", "150", "rocprofv3", "--kernel-trace", "--stats", "--output-format", "csv",
               "-d", td, "-o", "run", "--"] + _child_cmd(args, CHILD_STEPS)
        try:
            subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, check=True, timeout=180)
        except Exception:
            return None
        keep = os.environ.get("PQG_BENCH_PROF_DIR")  # keep the rocprofv3 output (profiles/)
        if keep:
            os.makedirs(keep, exist_ok=True)
            for pat, dst in (("*kernel_stats.csv", "rocprof_kernel_stats_%s.csv"),
                             ("*kernel_trace.csv", "rocprof_kernel_trace_%s.csv")):
                for f in glob.glob(os.path.join(td, "**", pat), recursive=True):
                    shutil.copy(f, os.path.join(keep, dst % args.config))
        rows = []
        for f in glob.glob(os.path.join(td, "**", "*kernel_trace.csv"), recursive=True):
            rows += list(csv.DictReader(open(f)))
    step = _last_steps(rows, "Dispatch_Id", "Kernel_Name")
    if not step:
        return None
    out = {}
    for r in step:
        k = out.setdefault(_kname(r["Kernel_Name"]), {"calls": 0, "ns": 0})
        k["calls"] += 1
        k["ns"] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    res = {k: {"avg_us": v["ns"] / v["calls"] / 1e3, "calls_per_step": v["calls"] / CHILD_STEPS,
               "us_per_step": v["ns"] / CHILD_STEPS / 1e3} for k, v in out.items()}
    if keep:
        with open(os.path.join(keep, "rocprof_kernel_steps_%s.csv" % args.config), "w") as f:
            f.write("# bench.py --config %s: the %d timed decode steps of the rocprofv3 --kernel-trace child run "
                    "(dispatches after the %d-th last %s), per kernel\n" % (args.config, CHILD_STEPS,
                                                                            CHILD_STEPS + 1,
                                                                            _step_end(sorted(rows, key=lambda r: int(r["Dispatch_Id"])), "Kernel_Name")))
            f.write("Name,CallsPerStep,AverageNs,NsPerStep\n")
            for k, v in sorted(res.items(), key=lambda kv: -kv[1]["us_per_step"]):
                f.write("%s,%g,%.0f,%.0f\n" % (k, v["calls_per_step"], v["avg_us"] * 1e3, v["us_per_step"] * 1e3))
    return res


def pmc_traffic(args):
    """HBM bytes per decode step of every kernel from rocprofv3 PMC counters,
    collected in separate passes (FETCH_SIZE, then WRITE_SIZE) over a short
    child run of this same bench, summed over each kernel's dispatches in the
    child's last CHILD_STEPS decode steps and divided by CHILD_STEPS.
    MI355X_MICROARCH.md: on gfx950 FETCH_SIZE reports half of a wide streaming
    read, so it is doubled.  Returns {kernel: {"fetch", "write",
    "dispatches_per_step"}} (bytes per step) or None."""
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile
    if not shutil.which("rocprofv3"):
        return None
    per = {}
    keep = os.environ.get("PQG_BENCH_PROF_DIR")
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as td:
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            out = os.path.join(td, ctr)
            cmd = ["timeout", "-s", "KILL", "120", "rocprofv3", "--pmc", ctr, "--output-format", "csv",
                   "-d", out, "-o", "run", "--"] + _child_cmd(args, CHILD_STEPS)
            try:
                subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, check=True, timeout=150)
            except Exception:
                return None
            rows = []
            for f in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
                if keep:
                    os.makedirs(keep, exist_ok=True)
                    shutil.copy(f, os.path.join(keep, "rocprof_pmc_%s_%s.csv" % (ctr.lower(), args.config)))
                rows += [r for r in csv.DictReader(open(f)) if r["Counter_Name"] == ctr]
            step = _last_steps(rows, "Dispatch_Id", "Kernel_Name")
            if not step:
                return None
            for r in step:
                k = per.setdefault(_kname(r["Kernel_Name"]), {})
                k.setdefault(ctr, []).append(float(r["Counter_Value"]) * 1024)  # kilobytes per dispatch
    res = {}
    for name, c in per.items():
        f, w = c.get("FETCH_SIZE", []), c.get("WRITE_SIZE", [])
        res[name] = {"fetch": 2 * sum(f) / CHILD_STEPS, "write": sum(w) / CHILD_STEPS,
                     "dispatches_per_step": max(len(f), len(w)) / CHILD_STEPS}
    return res or None


def gather_classes(args, rg0, rg1, decode_ms):
    """C2 only: the decode phase split by dictionary-index bit-width class,
    from the per-width rates tools/bw_sweep.sh measured (tools/gather_classes.json;
    single-width files, same kernel) and this shard's rows per width (row
    group i has bit width 1 + i % 20, tools/synth.py).  Names the share of the
    phase the L2-bound widths take, beside the gather ceilings."""
    ref = json.load(open(os.path.join(ROOT, "tools", "gather_classes.json")))
    rates = {int(k): v for k, v in ref["by_bit_width"].items()}
    known = sorted(rates)

    def rate(bw):
        if bw in rates:
            return rates[bw]
        lo = max(k for k in known if k < bw)
        hi = min(k for k in known if k > bw)
        return rates[lo] + (rates[hi] - rates[lo]) * (bw - lo) / (hi - lo)
    rows = {}
    for i in range(rg0, rg1):
        bw = 1 + i % 20
        rows[bw] = rows.get(bw, 0) + min(args.rg_rows, args.rows * max(1, args.gpus) - i * args.rg_rows)
    ms = {bw: n / (rate(bw) * 1e9) * 1e3 for bw, n in rows.items()}
    total = sum(ms.values())
    out = {"unit": "Gval/s", "source": ref["source"], "ceilings": ref["ceilings"], "classes": {}}
    for name, bws in ref["classes"].items():
        n = sum(rows.get(b, 0) for b in bws)
        t = sum(ms.get(b, 0.0) for b in bws)
        if n:
            out["classes"][name] = {"rows": n, "Gval_per_s": round(n / (t * 1e-3) / 1e9, 1),
                                    "predicted_ms": round(t, 4), "time_share": round(t / total, 3)}
    out["predicted_decode_ms"] = round(total, 4)
    out["measured_decode_ms"] = round(decode_ms, 4)
    return out


def segment_times(reader, rg0, rg1, decodes=6):
    """Every pipeline phase timed with HIP events (PQG_SEGMENT_TIMES=1) on a
    second batch of the same shard, outside the timed loop (each event adds a
    launch gap, so the timed loop brackets only the decode phase)."""
    os.environ["PQG_SEGMENT_TIMES"] = "1"
    try:
        b = reader.batch(rg0, rg1)
    finally:
        del os.environ["PQG_SEGMENT_TIMES"]
    try:
        b.decode()
        b.sync()
        b.kernel_times()
        for _ in range(decodes):
            b.decode()
        b.sync()
        return b.kernel_times()
    finally:
        b.close()


def e2e_rates(reader, rg0, rg1, stats, slice_counts=(2, 4, 8, 24), depth=8):
    """PCIe-inclusive rates (never `value`): the whole shard read through
    pqg_stream — the host worker plans and uploads slice k + 1 (pinned ring,
    PQG_UPLOAD_THREADS gather threads) while the GPU decodes slice k — timed
    from opening the stream to the last slice's sync; beside it the bare PCIe
    rates of the shard's input bytes from pinned host memory: one hipMemcpy,
    and 16 MiB hipMemcpyAsync chunks queued back to back (the yardstick is
    the faster of the two)."""
    hip = ctypes.CDLL("libamdhip64.so")
    n = int(stats["h2d_bytes"] or stats["input_bytes"])
    hbuf, dbuf, strm = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
    pcie, pcie_chunked = None, None
    if hip.hipHostMalloc(ctypes.byref(hbuf), ctypes.c_size_t(n), 0) == 0:
        if hip.hipMalloc(ctypes.byref(dbuf), ctypes.c_size_t(n)) == 0:
            ctypes.memset(hbuf, 1, n)
            hip.hipStreamCreate(ctypes.byref(strm))
            chunk = 16 << 20
            for _ in range(3):
                t = time.perf_counter()
                hip.hipMemcpy(dbuf, hbuf, ctypes.c_size_t(n), 1)  # hipMemcpyHostToDevice
                t = time.perf_counter() - t
                pcie = t if pcie is None else min(pcie, t)
                # the same bytes as 16 MiB asynchronous copies queued back to back
                t = time.perf_counter()
                for off in range(0, n, chunk):
                    hip.hipMemcpyAsync(ctypes.c_void_p(dbuf.value + off), ctypes.c_void_p(hbuf.value + off),
                                       ctypes.c_size_t(min(chunk, n - off)), 1, strm)
                hip.hipStreamSynchronize(strm)
                t = time.perf_counter() - t
                pcie_chunked = t if pcie_chunked is None else min(pcie_chunked, t)
            hip.hipStreamDestroy(strm)
            hip.hipFree(dbuf)
        hip.hipHostFree(hbuf)
    # slice sizes: small slices overlap more upload with decode; batches with
    # strings / lists pay a counting pass per slice whose time is set by their
    # longest pages, so they want few slices — the best of a few is reported
    best, per_best, tried = None, None, {}
    for slices in slice_counts:
        per = max(1, (rg1 - rg0 + slices - 1) // slices)
        if per in tried:
            continue
        bt = None
        for _ in range(2):  # the first pass also maps the file pages
            t = time.perf_counter()
            with reader.stream(rg0, rg1, per, None, depth) as st:
                for b in st:
                    b.sync()
            t = time.perf_counter() - t
            bt = t if bt is None else min(bt, t)
        tried[per] = round(bt * 1e3, 2)
        if best is None or bt < best:
            best, per_best = bt, per
    # the best slice size again with the first two slices a quarter / half of
    # it (pqgpu.STREAM_RAMP: the first decode starts after a short upload)
    import pqgpu  # (sys.path set by main)
    if per_best > 1:
        bt = None
        for _ in range(2):
            t = time.perf_counter()
            with reader.stream(rg0, rg1, per_best, None, depth, pqgpu.STREAM_RAMP) as st:
                for b in st:
                    b.sync()
            t = time.perf_counter() - t
            bt = t if bt is None else min(bt, t)
        tried["%d+ramp" % per_best] = round(bt * 1e3, 2)
        if bt < best:
            best, per_best = bt, "%d+ramp" % per_best
    out = {"stream_ms": round(best * 1e3, 2), "stream_rgs_per_slice": per_best, "stream_depth": depth,
           "stream_ms_by_rgs_per_slice": tried,
           "GBps_stream_incl_plan_and_h2d": round(stats["output_bytes"] / best / 1e9, 1),
           "h2d_bytes": n}
    if pcie:
        out["pcie_only_ms"] = round(pcie * 1e3, 2)
        out["pcie_only_GBps_in"] = round(n / pcie / 1e9, 1)
        out["pcie_chunked_ms"] = round(pcie_chunked * 1e3, 2)
        out["pcie_chunked_GBps_in"] = round(n / pcie_chunked / 1e9, 1)
        # the decoded-bytes rate a pure upload of the shard's input would allow
        # (the faster of one copy and 16 MiB async chunks: the yardstick)
        yard = min(pcie, pcie_chunked)
        out["GBps_pcie_only_decoded_equiv"] = round(stats["output_bytes"] / yard / 1e9, 1)
        out["stream_vs_pcie_only"] = round(yard / best, 3)
    return out


def parity_check(reader, rg0, rg1, threads):
    """Every row group of the rank's shard decoded again on the GPU (one
    batch per row group, outside the timed region) and compared bit-exactly,
    buffer by buffer, with the oracle's decode of the same row group (oracle
    decodes run on `threads` host threads ahead of the GPU comparisons)."""
    import concurrent.futures as cf
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    cols = reader.Columns()
    o = oracle.File(open(reader.path, "rb").read())
    keys = ("values", "validity", "list_offsets", "list_validity", "str_offsets")

    def want(rg):
        return [o.decode(i, rg, rg + 1) for i in range(len(cols))]

    ok, t0 = 0, time.perf_counter()
    with cf.ThreadPoolExecutor(max(1, threads)) as ex:
        pending = {}
        nxt = rg0
        for rg in range(rg0, rg1):
            while nxt < rg1 and nxt < rg + 2 * max(1, threads):
                pending[nxt] = ex.submit(want, nxt)
                nxt += 1
            b = reader.batch(rg, rg + 1, list(range(len(cols))))
            try:
                b.decode()
                b.sync()
                ref = pending.pop(rg).result()
                for i, info in enumerate(cols):
                    got = b.column(i)
                    for k in keys:
                        if k == "validity" and info["max_def"] == 0:
                            continue
                        if k in ("list_offsets", "list_validity") and info["max_rep"] != 1:
                            continue
                        if not np.array_equal(got[k], ref[i][k]):
                            for f in pending.values():
                                f.cancel()
                            return False, "MISMATCH in row group %d leaf %s buffer %s" % (rg, info["name"], k)
            finally:
                b.close()
            ok += 1
    return True, "per-RG batches bit-exact vs oracle: %d/%d row groups, %d leaves, every buffer (%.1f s)" % (
        ok, rg1 - rg0, len(cols), time.perf_counter() - t0)


def timed_batch_parity(batch, reader, rg0, rg1, threads):
    """The timed batch itself — the buffers its last timed decode left on the
    device, every selected leaf over the whole shard [rg0, rg1) — copied back
    and compared bit-exactly with the oracle's decode of the same row-group
    range (oracle/pqref.c; type_dict.go:39-59, chunk_reader.go:380-402).  The
    per-row-group batches of parity_check take other kernel routes (a lone
    row group's big dictionary may run k_expand_wg, the XCD dealing differs),
    so this is the check that pins the headline's own bytes.  Oracle decodes
    run on `threads` host threads, a few leaves ahead of the GPU copies.
    Returns (ok, text)."""
    import concurrent.futures as cf
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    cols = reader.Columns()
    o = oracle.File(open(reader.path, "rb").read())
    keys = ("values", "validity", "list_offsets", "list_validity", "str_offsets")
    leaves = list(batch.leaves)
    t0 = time.perf_counter()
    window = max(1, min(len(leaves), threads, 4))
    with cf.ThreadPoolExecutor(window) as ex:
        pending = {}
        for i, leaf in enumerate(leaves):
            for j in range(i, min(len(leaves), i + window)):
                if j not in pending:
                    pending[j] = ex.submit(o.decode, leaves[j], rg0, rg1)
            ref = pending.pop(i).result()
            got = batch.column(i)
            info = cols[leaf]
            for k in keys:
                if k == "validity" and info["max_def"] == 0:
                    continue
                if k in ("list_offsets", "list_validity") and info["max_rep"] != 1:
                    continue
                if got[k].size != ref[k].size or not np.array_equal(got[k], ref[k]):
                    for f in pending.values():
                        f.cancel()
                    return False, "MISMATCH in the timed batch: leaf %s buffer %s (%d vs %d bytes)" % (
                        info["name"], k, got[k].size, ref[k].size)
            for k in ("slots", "str_bytes"):
                if got[k] != ref[k]:
                    return False, "MISMATCH in the timed batch: leaf %s count %s" % (info["name"], k)
            del got, ref
    return True, "timed batch bit-exact vs oracle (%d RGs, %d leaves, every buffer, %.1f s)" % (
        rg1 - rg0, len(leaves), time.perf_counter() - t0)


def pyarrow_baseline(path, cores, out_bytes, total_rows, budget_s=4.0):
    """pq.read_table(use_threads=True) on the same file, row group by row
    group until ~budget_s (an independent CPU decoder beside
    the oracle port); decoded bytes counted as the GPU counts them (the
    shard's B_out scaled by the rows read).  None without pyarrow."""
    try:
        import pyarrow as pa
        import pyarrow.parquet as pq
    except Exception:
        return None
    pa.set_cpu_count(cores)
    pa.set_io_thread_count(cores)
    pf = pq.ParquetFile(path)
    n = pf.num_row_groups
    rows, rgs, t0 = 0, 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        k = rgs % n
        t = pf.read_row_groups([k], use_threads=True)
        rows += t.num_rows
        rgs += 1
        del t
    dt = time.perf_counter() - t0
    return {"value": round(out_bytes * rows / total_rows / dt / 1e9, 3), "unit": "GB/s", "threads": cores,
            "pyarrow": pa.__version__,
            "sample": "ParquetFile.read_row_groups([rg], use_threads=True), %d row-group reads (%d rows), %.1f s"
                      % (rgs, rows, dt)}


def spawn_ranks(args):
    """`bench.py --gpus N` without an external launcher: start N rank
    processes (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set) before anything
    touches the GPU, wait for all, and exit with the worst status.  Rank 0's
    JSON line is the job's line."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    rc = 0
    for p in procs:
        rc = max(rc, abs(p.wait()))
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=sorted(synth.DEFAULTS))
    ap.add_argument("--rows", type=int, default=0, help="rows per GPU (default: the config's)")
    ap.add_argument("--rg-rows", type=int, default=0, help="rows per row group (default: the config's)")
    ap.add_argument("--file", default=None)
    ap.add_argument("--cpu-budget", type=float, default=8.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-prof", action="store_true", help="skip the rocprofv3 child runs (kernel trace, PMC)")
    ap.add_argument("--no-pmc", action="store_true", help="(compat) same as --no-prof")
    ap.add_argument("--no-parity", action="store_true", help="skip the whole-shard oracle comparison")
    ap.add_argument("--child", action="store_true", help="internal: a profiled child run (timed loop only)")
    ap.add_argument("--allgather", action="store_true",
                    help="N > 1: time the optional column all-gather and gather-to-root (RCCL)")
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="N > 1: process group backend for the barrier / max-time reduction (gloo: ranks may "
                         "share a GPU, as in the CPU-box test)")
    ap.add_argument("--bw", type=int, default=0, help="analysis: one dictionary bit width for every row group")
    args = ap.parse_args()
    args.rows = args.rows or synth.DEFAULTS[args.config][0]
    args.rg_rows = args.rg_rows or synth.DEFAULTS[args.config][1]
    if args.child:
        args.no_cpu = args.no_prof = True

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    dist, device = None, 0
    if world > 1:
        import torch
        import torch.distributed as dist
        ndev = max(1, torch.cuda.device_count())  # counts devices without initialising HIP
        device = local % ndev
        if args.dist_backend == "nccl":
            if local >= ndev:
                sys.exit("bench.py: %d local ranks on %d GPUs need --dist-backend gloo" % (world, ndev))
            torch.cuda.set_device(device)
        dist.init_process_group(args.dist_backend)

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

    ctx = pqgpu.Context(device)
    reader = pqgpu.FileReader(path, ctx=ctx)
    reader.path = path
    sizes = [reader.RowGroupCost(i) for i in range(reader.RowGroupCount())]  # balanced by decode cost
    rg0, rg1 = pqgpu.plan_row_group_shards(sizes, world)[rank]
    # first use: HIP runtime, pinned ring, device buffers and the kernels' code
    # objects (loaded at their first launch) set up outside every timing
    wb = reader.batch(rg0, rg1)
    wb.decode()
    wb.sync()
    wb.close()
    # one-shot PCIe-inclusive time (not `value`): host plan + H2D upload + one
    # decode, to the decode's sync (the upload's DMAs finish inside it).  The
    # median of five trials is the headline; min / max and every trial's stage
    # breakdown (pqg_batch_create's host stages, then decode launch to sync)
    # are kept in the line
    oneshot_trials, oneshot_stages = [], []
    for _ in range(5):
        t0 = time.perf_counter()
        b1 = reader.batch(rg0, rg1)
        t1 = time.perf_counter()
        b1.decode()
        t2 = time.perf_counter()
        b1.sync()
        t3 = time.perf_counter()
        oneshot_trials.append(t3 - t0)
        st = b1.stats()
        oneshot_stages.append({k: round(st[k], 2) for k in ("create_plan_ms", "create_alloc_ms", "create_upload_ms",
                                                            "upload_gather_ms", "upload_wait_ms", "create_tables_ms")})
        oneshot_stages[-1].update({"create_ms": round((t1 - t0) * 1e3, 2), "decode_launch_ms": round((t2 - t1) * 1e3, 2),
                                   "sync_ms": round((t3 - t2) * 1e3, 2)})
        b1.close()
    t_oneshot = sorted(oneshot_trials)[len(oneshot_trials) // 2]
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
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipDeviceSynchronize()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    hip.hipDeviceSynchronize()
    barrier()
    dt = time.perf_counter() - t0
    batch.sync()  # raises if any page failed to decode
    decode_ms = batch.kernel_times()  # HIP-event time of the decode phase during the timed steps
    out_b, in_b = stats["output_bytes"], stats["input_bytes"]
    job_out = out_b
    if dist is not None:
        import torch
        dev = torch.device("cuda", device) if args.dist_backend == "nccl" else torch.device("cpu")
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)  # the slowest rank sets the job time
        dt = float(t.item())
        nb = torch.tensor([out_b], dtype=torch.float64, device=dev)
        dist.all_reduce(nb, op=dist.ReduceOp.SUM)  # every rank's decoded bytes
        job_out = float(nb.item())
    per_step = dt / args.steps
    value = job_out * args.steps / dt / 1e9

    allgather = None
    if dist is not None and args.allgather and args.dist_backend == "nccl":
        import torch
        import pqgather
        dev = torch.device("cuda", device)
        shard = pqgather.shard_tensors(batch, 0, dev)
        torch.cuda.synchronize(dev)
        barrier()
        ta = time.perf_counter()
        col = pqgather.allgather_column(shard)
        torch.cuda.synchronize(dev)
        ta = time.perf_counter() - ta
        gb = sum(v.numel() * v.element_size() for v in col.values() if hasattr(v, "numel")) / 1e9
        del col
        # the all-to-one form: the whole column on rank 0 only
        barrier()
        tr = time.perf_counter()
        col = pqgather.gather_column_to(shard, 0)
        torch.cuda.synchronize(dev)
        tr = time.perf_counter() - tr
        del col
        tr_max = torch.tensor([tr], dtype=torch.float64, device=dev)
        dist.all_reduce(tr_max, op=dist.ReduceOp.MAX)
        tr = float(tr_max.item())
        allgather = {"leaf": 0, "GB_per_rank": round(gb, 4), "ms": round(ta * 1e3, 3), "GBps_per_rank": round(gb / ta, 1),
                     "gather_to_root_ms": round(tr * 1e3, 3), "gather_to_root_GBps": round(gb / tr, 1)}
    parity = None
    if not (args.child or args.no_parity):
        # the timed batch's own output, on every rank, before it is closed
        ok, txt = timed_batch_parity(batch, reader, rg0, rg1, cpu_cores()[0])
        if ok:
            ok2, txt2 = parity_check(reader, rg0, rg1, cpu_cores()[0])
            ok, txt = ok and ok2, txt + " + " + txt2
        if dist is not None:
            import torch
            dev = torch.device("cuda", device) if args.dist_backend == "nccl" else torch.device("cpu")
            f = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
            dist.all_reduce(f, op=dist.ReduceOp.MIN)  # every rank's shard must be bit-exact
            ranks_ok = int(f.item()) == 1
            txt = ("all %d ranks: " % world if ranks_ok else "MISMATCH on some rank; rank %d: " % rank) + txt
            ok = ok and ranks_ok
        parity = {"ok": ok, "text": txt}
    batch.close()
    if args.child:
        if dist is not None:
            dist.destroy_process_group()
        return

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
                   "job_B_out": job_out,
                   "pages": stats["data_pages"], "dict_pages": stats["dict_pages"],
                   "B_in": in_b, "B_out": out_b, "staged": stats["staged_bytes"],
                   "snappy_in": stats["snappy_in_bytes"],
                   "decode_phase_ms_timed": {k: round(v, 4) for k, v in decode_ms.items()},
                   # PCIe-inclusive rate (not `value`): host planning + H2D upload + one
                   # decode, timed to its sync (batch_create_ms alone returns before the
                   # upload's DMAs end)
                   "e2e": {"batch_create_ms": round(t_create * 1e3, 2),
                           "oneshot_ms": round(t_oneshot * 1e3, 2),
                           "oneshot_ms_min_median_max": [round(min(oneshot_trials) * 1e3, 2), round(t_oneshot * 1e3, 2),
                                                         round(max(oneshot_trials) * 1e3, 2)],
                           "oneshot_trials_ms": [round(t * 1e3, 2) for t in oneshot_trials],
                           "oneshot_stages": oneshot_stages,
                           "GBps_incl_plan_and_h2d": round(out_b / t_oneshot / 1e9, 1)},
                   "parallelism": "row-group shards, one process per GPU, no data-path collective"
                                  + ("" if world == 1 else " (%s for the barrier / time reduction)"
                                     % args.dist_backend)},
    }
    if allgather:
        line["config"]["allgather"] = allgather
    if parity is not None:
        line["config"]["parity"] = parity["text"]
        line["config"]["parity_ok"] = parity["ok"]
    if rank == 0 and world == 1:
        seg = segment_times(reader, rg0, rg1)
        line["config"]["phase_ms"] = {k: round(v, 4) for k, v in seg.items()}
        dom = max(seg, key=seg.get)
        ach = phase_bytes(dom, stats) / (seg[dom] * 1e-3) / 1e9
        # the dominant phase's roofline: live HIP events around the phase;
        # beside it the same bytes over the phase's kernels' per-step time in
        # the bench's own rocprofv3 trace (profiles/.../rocprof_kernel_steps_*)
        line["roofline"] = {"bound": "hbm", "kernel": dom, "phase": dom, "phase_ms": round(seg[dom], 4),
                            "algorithmic_bytes": phase_bytes(dom, stats),
                            "achieved": round(ach, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                            "frac": round(ach / HBM_PEAK_GBPS, 4), "traffic": None,
                            "pipeline_frac": round((in_b + out_b) / per_step / 1e9 / HBM_PEAK_GBPS, 4)}
        if args.config == "c2" and not args.bw and "k_decode+k_expand" in seg:
            try:
                line["roofline"]["gather_classes"] = gather_classes(args, rg0, rg1, seg["k_decode+k_expand"])
            except Exception as e:  # (analysis figure only)
                line["roofline"]["gather_classes"] = {"error": str(e)}
        trace = None if args.no_prof or args.no_pmc else kernel_trace(args)
        if trace:
            line["config"]["kernel_trace_us_per_step"] = {
                k: [round(v["us_per_step"], 2), v["calls_per_step"]]
                for k, v in sorted(trace.items(), key=lambda kv: -kv[1]["us_per_step"])}
            mine = {k: v for k, v in trace.items() if k.startswith(PHASE_KERNELS[dom])}
            if mine:
                kern = max(mine, key=lambda k: mine[k]["us_per_step"])
                tsum = sum(v["us_per_step"] for v in mine.values())
                line["roofline"].update({
                    "kernel": kern, "kernel_avg_us": round(mine[kern]["avg_us"], 2),
                    "kernel_calls_per_step": mine[kern]["calls_per_step"],
                    "phase_kernels_us_per_step": round(tsum, 2),
                    # equals `frac` when the phase is one kernel on one stream;
                    # lower when its kernels overlap on side streams
                    "frac_from_trace": round(phase_bytes(dom, stats) / (tsum * 1e-6) / 1e9 / HBM_PEAK_GBPS, 4)})
        if not (args.no_prof or args.no_pmc):
            pmc = pmc_traffic(args)
            if pmc:
                line["config"]["pmc_MB_per_step"] = {k: {"fetch": round(v["fetch"] / 1e6, 1),
                                                         "write": round(v["write"] / 1e6, 1),
                                                         "dispatches": v["dispatches_per_step"]}
                                                     for k, v in sorted(pmc.items())}
                ks = [k for k in pmc if k.startswith(PHASE_KERNELS[dom])]
                if ks:
                    tr = sum(pmc[k]["fetch"] + pmc[k]["write"] for k in ks)
                    line["roofline"]["traffic"] = round(tr / 1e6, 1)
                    line["roofline"]["traffic_unit"] = ("MB per decode step, summed over every dispatch of the "
                                                        "phase's kernels (FETCH_SIZE x 2 + WRITE_SIZE)")
                    line["roofline"]["traffic_vs_algorithmic"] = round(tr / phase_bytes(dom, stats), 3)
        line["config"]["e2e"].update(e2e_rates(reader, rg0, rg1, stats))
    if "roofline" not in line:
        # N > 1: the decode phase, HIP events over the timed steps (per rank)
        dms = sum(decode_ms.values())
        if dms > 0:
            ach = (in_b + out_b) / (dms * 1e-3) / 1e9
            line["roofline"] = {"bound": "hbm", "kernel": "k_decode+k_expand", "phase": "k_decode+k_expand",
                                "phase_ms": round(dms, 4), "achieved": round(ach, 1), "peak": HBM_PEAK_GBPS,
                                "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBPS, 4), "traffic": None,
                                "pipeline_frac": round((in_b + out_b) / per_step / 1e9 / HBM_PEAK_GBPS, 4)}
    if rank == 0 and world == 1 and not args.no_cpu:
        line["cpu_baseline"] = cpu_baseline(path, args.cpu_budget)
        pa_line = pyarrow_baseline(path, line["cpu_baseline"]["cores"], out_b, stats_rows(reader, rg0, rg1))
        if pa_line:
            line["cpu_baseline"]["pyarrow_read_table"] = pa_line
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def stats_rows(reader, rg0, rg1):
    return sum(reader.RowGroupNumRows(i) for i in range(rg0, rg1))


if __name__ == "__main__":
    main()
