"""N > 1 path on CPU: row-group shards over world_size 2 ranks with gloo.

The decode path has no collective (row groups are independent,
chunk_reader.go:221); what the multi-GPU bench adds is (1) the shard plan,
(2) max-over-ranks timing and (3) whole-job aggregation of decoded bytes.
These tests run that exact logic with 2 gloo ranks on 127.0.0.1, each rank
decoding its shard with the CPU oracle (the checker), and check that the
shards tile the file and that the aggregated result equals the whole-file
decode.
"""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_plan_row_group_shards_tiles_and_balances():
    import pqgpu
    sizes = [5, 1, 1, 1, 9, 2, 2, 3]
    for world in (1, 2, 3, 4, 8, 11):
        sh = pqgpu.plan_row_group_shards(sizes, world)
        assert len(sh) == world
        assert sh[0][0] == 0 and sh[-1][1] == len(sizes)
        for (a0, a1), (b0, b1) in zip(sh, sh[1:]):
            assert a1 == b0 and a0 <= a1
        if world <= len(sizes):
            assert all(b > a for a, b in sh)
    # balanced: equal sizes split evenly
    sh = pqgpu.plan_row_group_shards([1] * 96, 8)
    assert [b - a for a, b in sh] == [12] * 8


def test_cost_balanced_shards_c2_shape(tmp_path):
    """plan_row_group_shards over FileReader.RowGroupCost: C2's row groups
    (dictionary bit width 1 + i % 20) cost by their bit width, not by their
    bytes (a bit-width-20 row group carries a 4 MiB dictionary page but its
    gathers, not its bytes, are the cost).  The cost estimate grows with the
    bit width past the LDS-resident sizes, and the cost-balanced plan's
    heaviest shard is no heavier (in cost) than the byte-balanced plan's."""
    pytest.importorskip("pyarrow")
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import synth
    import pqgpu
    path = str(tmp_path / "c2_cost.parquet")
    synth.make("c2", path, 40 * 20000, 20000)  # 40 row groups: bit widths 1..20 twice
    r = pqgpu.FileReader(path)
    n = r.RowGroupCount()
    assert n == 40
    cost = [r.RowGroupCost(i) for i in range(n)]
    size = [r.RowGroupByteSize(i) for i in range(n)]
    assert all(c > 0 for c in cost)
    assert r.RowGroupCost(n) < 0 and r.RowGroupCost(-1) < 0
    # bit width b + 1 at row group b: big dictionaries cost more per row
    assert cost[19] > cost[11] * 1.5 and cost[15] > cost[5] * 1.5
    assert abs(cost[3] - cost[23]) < 0.05 * cost[3]  # same width, same cost
    for world in (2, 3, 4, 8):
        by_cost = pqgpu.plan_row_group_shards(cost, world)
        by_size = pqgpu.plan_row_group_shards(size, world)
        worst = lambda plan: max(sum(cost[a:b]) for a, b in plan)
        assert worst(by_cost) <= worst(by_size) * 1.0001, (world, by_cost, by_size)
        assert by_cost[0][0] == 0 and by_cost[-1][1] == n


def test_cost_prices_dictionary_at_data_page_offset():
    """A writer that leaves dictionary_page_offset unset puts the dictionary
    page at data_page_offset: RowGroupCost still finds it there and prices
    the gathers by its bit width (the same cost as with the field set), and
    both layouts decode alike on the oracle."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle
    import pqgpu
    import pqwrite
    rng = np.random.default_rng(44)
    dn, n = 20000, 200000  # bit width 15: L2 gathers
    keys = rng.integers(0, dn, n)
    dvals = rng.integers(-2**31, 2**31, dn).astype("<i4").tobytes()
    rg = {"dict_page": dvals, "dict_count": dn, "pages": [(n, None, bytes([15]) + pqwrite.hybrid_bitpacked(keys, 15))]}
    with_field = pqwrite.write_row_groups([rg], ptype=1, encoding=8)
    without = pqwrite.write_row_groups([rg], ptype=1, encoding=8, dict_offset_field=False)
    c1 = pqgpu.FileReader(with_field).RowGroupCost(0)
    c2 = pqgpu.FileReader(without).RowGroupCost(0)
    assert c1 > 0 and abs(c1 - c2) < 1e-6 * c1, (c1, c2)
    assert c1 > len(with_field) / 2000.0 * 1.5  # the gathers, not only the bytes
    a = oracle.File(with_field).decode(0)["values"].view(np.int32)
    b = oracle.File(without).decode(0)["values"].view(np.int32)
    assert np.array_equal(a, b) and np.array_equal(a, np.frombuffer(dvals, "<i4")[keys])


def _rank_main(rank, world, port, path, out_dir):
    import torch
    import torch.distributed as dist
    sys.path[:0] = [os.path.join(ROOT, "parquet-go_amd"), os.path.join(ROOT, "oracle")]
    import oracle
    import pqgpu
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    data = open(path, "rb").read()
    r = pqgpu.FileReader(data)  # host-side metadata only: no GPU needed
    sizes = [r.RowGroupCost(i) for i in range(r.RowGroupCount())]
    rg0, rg1 = pqgpu.plan_row_group_shards(sizes, world)[rank]
    import time
    t0 = time.perf_counter()
    got = oracle.File(data).decode(0, rg0, rg1)
    dt = time.perf_counter() - t0
    vals = np.asarray(got["values"]).view(np.uint8)
    t = torch.tensor([dt], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)  # the bench's max-over-ranks time
    nb = torch.tensor([vals.size], dtype=torch.int64)
    dist.all_reduce(nb, op=dist.ReduceOp.SUM)  # whole-job decoded bytes
    parts = [None] * world
    dist.all_gather_object(parts, (rg0, rg1, vals.tobytes()))
    if rank == 0:
        np.save(os.path.join(out_dir, "agg.npy"),
                np.frombuffer(b"".join(p[2] for p in parts), np.uint8))
        with open(os.path.join(out_dir, "meta.txt"), "w") as f:
            f.write("%d %f %s\n" % (int(nb.item()), float(t.item()), ";".join("%d-%d" % p[:2] for p in parts)))
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_rank_gloo_shards_match_whole_file(tmp_path):
    pa = pytest.importorskip("pyarrow")
    import pyarrow.parquet as pq
    torch = pytest.importorskip("torch")
    import torch.multiprocessing as mp
    import oracle
    rng = np.random.default_rng(7)
    n = 60000
    path = str(tmp_path / "shards.parquet")
    keys = rng.integers(0, 300, n)
    dvals = rng.permutation(1 << 16)[:300].astype(np.int32)
    pq.write_table(pa.table({"v": pa.array(dvals[keys])}), path, row_group_size=7000, compression="snappy",
                   use_dictionary=True)
    world = 2
    mp.spawn(_rank_main, args=(world, _free_port(), path, str(tmp_path)), nprocs=world, join=True)
    agg = np.load(str(tmp_path / "agg.npy"))
    nbytes, tmax, shards = open(str(tmp_path / "meta.txt")).read().split()
    whole = np.asarray(oracle.File(open(path, "rb").read()).decode(0)["values"]).view(np.uint8)
    assert int(nbytes) == whole.size == agg.size
    assert np.array_equal(agg, whole)
    assert float(tmax) > 0
    (a0, a1), (b0, b1) = [tuple(map(int, s.split("-"))) for s in shards.split(";")]
    assert a0 == 0 and a1 == b0 and b1 == pq.ParquetFile(path).num_row_groups


def _gather_main(rank, world, port, path, leaf, out_dir, root=-1):
    import torch
    import torch.distributed as dist
    sys.path[:0] = [os.path.join(ROOT, "parquet-go_amd"), os.path.join(ROOT, "oracle")]
    import oracle
    import pqgather
    import pqgpu
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    data = open(path, "rb").read()
    r = pqgpu.FileReader(data)
    sizes = [r.RowGroupByteSize(i) for i in range(r.RowGroupCount())]
    rg0, rg1 = pqgpu.plan_row_group_shards(sizes, world)[rank]
    o = oracle.File(data)
    got = o.decode(leaf, rg0, rg1)  # this rank's shard (the checker stands in for the GPU)
    info = o.leaves()[leaf]
    # buffers present by schema (as the GPU column view has them), even when the shard is empty
    present = {"validity": info["max_def"] > 0, "list_offsets": info["max_rep"] == 1,
               "list_validity": info["max_rep"] == 1, "str_offsets": info["physical_type"] == 6}

    def t(name, dt):
        if not present[name]:
            return None
        a = got[name]
        if name == "list_offsets" and a.size == 0:
            a = np.zeros(4, np.uint8)  # rows + 1 offsets of an empty shard
        if name == "str_offsets" and a.size == 0:
            a = np.zeros(8, np.uint8)
        return torch.from_numpy(a.view(dt).copy())

    shard = {"slots": int(got["slots"]), "rows": int(got["rows"]), "values": torch.from_numpy(got["values"].copy()),
             "validity": t("validity", np.uint8), "list_offsets": t("list_offsets", np.int32),
             "list_validity": t("list_validity", np.uint8), "str_offsets": t("str_offsets", np.int64)}
    if root < 0:
        col = pqgather.to_numpy(pqgather.allgather_column(shard))
        if rank == world - 1:
            np.savez(os.path.join(out_dir, "gathered.npz"), **{k: np.asarray(v) for k, v in col.items()})
    else:
        col = pqgather.gather_column_to(shard, root)
        assert (col is None) == (rank != root), (rank, root)
        if rank == root:
            col = pqgather.to_numpy(col)
            np.savez(os.path.join(out_dir, "gathered.npz"), **{k: np.asarray(v) for k, v in col.items()})
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("name,leaf,world", [("c4_list_str", 0, 2), ("c4_list_str", 1, 3), ("c3_delta_v2", 1, 2),
                                             ("plain_strings", 0, 3), ("c2_dict_bw8", 0, 2),
                                             # more ranks than row groups: the last ranks hold empty shards
                                             ("c4_list_str", 0, 4), ("gzip_int64", 0, 5)])
def test_allgather_column_gloo(tmp_path, name, leaf, world):
    """The optional all-gather over gloo: every rank ends with
    the whole column, equal to the whole-file decode (bitmaps re-packed at odd
    shard boundaries, list / string offsets rebased)."""
    pytest.importorskip("torch")
    import torch.multiprocessing as mp
    import oracle
    path = os.path.join(GOLDEN, name + ".parquet")
    mp.spawn(_gather_main, args=(world, _free_port(), path, leaf, str(tmp_path)), nprocs=world, join=True)
    got = np.load(str(tmp_path / "gathered.npz"))
    whole = oracle.File(open(path, "rb").read()).decode(leaf)
    assert int(got["slots"]) == whole["slots"] and int(got["rows"]) == whole["rows"]
    info = oracle.File(open(path, "rb").read()).leaves()[leaf]
    for k in ("values", "validity", "list_offsets", "list_validity", "str_offsets"):
        if k == "validity" and info["max_def"] == 0:
            continue  # a required column has no bitmap on the GPU (the oracle's is all ones)
        assert np.array_equal(got[k].view(np.uint8).ravel(), whole[k]), k


@pytest.mark.timeout(300)
@pytest.mark.parametrize("name,leaf,world,root", [("c4_list_str", 0, 2, 0), ("c4_list_str", 1, 3, 2),
                                                  ("c3_delta_v2", 1, 3, 1), ("plain_strings", 0, 2, 1),
                                                  ("c2_dict_bw8", 0, 3, 0),
                                                  # more ranks than row groups: empty shards send nothing
                                                  ("c4_list_str", 0, 5, 3), ("gzip_int64", 0, 5, 0)])
def test_gather_column_to_root_gloo(tmp_path, name, leaf, world, root):
    """The all-to-one materialisation over gloo: only the
    root ends with the whole column, equal to the whole-file decode."""
    pytest.importorskip("torch")
    import torch.multiprocessing as mp
    import oracle
    path = os.path.join(GOLDEN, name + ".parquet")
    mp.spawn(_gather_main, args=(world, _free_port(), path, leaf, str(tmp_path), root), nprocs=world, join=True)
    got = np.load(str(tmp_path / "gathered.npz"))
    o = oracle.File(open(path, "rb").read())
    whole, info = o.decode(leaf), o.leaves()[leaf]
    assert int(got["slots"]) == whole["slots"] and int(got["rows"]) == whole["rows"]
    for k in ("values", "validity", "list_offsets", "list_validity", "str_offsets"):
        if k == "validity" and info["max_def"] == 0:
            continue
        assert np.array_equal(got[k].view(np.uint8).ravel(), whole[k]), k


def _gpu_shard_main(rank, world, port, path, leaf, out_dir):
    import torch
    import torch.distributed as dist
    sys.path[:0] = [os.path.join(ROOT, "parquet-go_amd")]
    import pqgather
    import pqgpu
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    r = pqgpu.FileReader(path)
    sizes = [r.RowGroupByteSize(i) for i in range(r.RowGroupCount())]
    rg0, rg1 = pqgpu.plan_row_group_shards(sizes, world)[rank]
    b = r.batch(rg0, rg1, [leaf])  # this rank's shard, decoded by libpqgpu.so on cuda:0
    b.decode()
    dev = torch.device("cuda", 0)
    shard = pqgather.shard_tensors(b, 0, dev)  # device-to-device copies out of the batch
    b.close()
    host = {k: (v.cpu() if hasattr(v, "cpu") else v) for k, v in shard.items()}  # gloo gathers host tensors
    col = pqgather.to_numpy(pqgather.allgather_column(host))
    if rank == 0:
        np.savez(os.path.join(out_dir, "gathered.npz"), **{k: np.asarray(v) for k, v in col.items()})
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.timeout(300)
@pytest.mark.parametrize("name,leaf,world", [("c4_list_str", 0, 2), ("c4_list_str", 1, 4), ("c3_delta_v2", 1, 2)])
def test_gpu_shards_allgather(tmp_path, name, leaf, world):
    """The N > 1 data path with the product decoder: each rank plans its
    row-group shard, decodes it with libpqgpu.so on the (one) GPU, copies the
    buffers device to device (pqgather.shard_tensors) and all-gathers them;
    the result equals the whole-file oracle decode.  `world` ranks share
    cuda:0 here; the 8-GPU bench runs one rank per GPU over RCCL."""
    import torch.multiprocessing as mp
    import oracle
    path = os.path.join(GOLDEN, name + ".parquet")
    mp.spawn(_gpu_shard_main, args=(world, _free_port(), path, leaf, str(tmp_path)), nprocs=world, join=True)
    got = np.load(str(tmp_path / "gathered.npz"))
    o = oracle.File(open(path, "rb").read())
    whole, info = o.decode(leaf), o.leaves()[leaf]
    assert int(got["slots"]) == whole["slots"]
    for k in ("values", "validity", "list_offsets", "list_validity", "str_offsets"):
        if k == "validity" and info["max_def"] == 0:
            continue
        assert np.array_equal(got[k].view(np.uint8).ravel(), whole[k]), k


def _bench_line(tmp_path, gpus, path, config="c1", parity=False):
    import json
    import subprocess
    env = dict(os.environ, TMPDIR=str(tmp_path))
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--config", config,
                          "--rows", "300000", "--rg-rows", "50000", "--steps", "3", "--warmup", "1", "--file", path,
                          "--no-prof", "--no-cpu", "--dist-backend", "gloo"] + ([] if parity else ["--no-parity"]),
                         env=env, capture_output=True, text=True, timeout=240, check=True)
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout + out.stderr
    return json.loads(lines[0])


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_bench_gpus_2_spawns_two_ranks(tmp_path):
    """`bench.py --gpus 2` without a launcher starts two rank processes
    (sharing cuda:0 over gloo here; one GPU each over RCCL on a node): the
    line reports n_gpus 2 and the job's decoded bytes equal a 1-rank run's."""
    pytest.importorskip("pyarrow")
    pytest.importorskip("torch")
    path = str(tmp_path / "c1_small.parquet")
    two = _bench_line(tmp_path, 2, path)
    one = _bench_line(tmp_path, 1, path)
    assert two["n_gpus"] == 2 and one["n_gpus"] == 1
    assert two["config"]["job_B_out"] == one["config"]["job_B_out"] == one["config"]["B_out"]
    assert 0 < two["config"]["B_out"] < one["config"]["B_out"]  # rank 0 decoded its shard only
    assert two["value"] > 0


@pytest.mark.gpu
@pytest.mark.timeout(300)
@pytest.mark.parametrize("config", ["c2", "c4"])
def test_bench_timed_batch_parity_every_rank(tmp_path, config):
    """bench.py compares the timed batch's own buffers (whole shard, every
    leaf) with the oracle on every rank and all-reduces the verdict."""
    pytest.importorskip("pyarrow")
    pytest.importorskip("torch")
    path = str(tmp_path / ("%s_small.parquet" % config))
    for gpus in (2, 1):
        line = _bench_line(tmp_path, gpus, path, config, parity=True)
        assert line["config"]["parity_ok"] is True, line["config"]["parity"]
        assert "timed batch bit-exact" in line["config"]["parity"]
        if gpus == 2:
            assert line["config"]["parity"].startswith("all 2 ranks")


def _gpu_rccl_main(rank, world, port, path, leaf, out_dir, mode="all"):
    import torch
    import torch.distributed as dist
    sys.path[:0] = [os.path.join(ROOT, "parquet-go_amd")]
    import pqgather
    import pqgpu
    torch.cuda.set_device(rank)
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    r = pqgpu.FileReader(path)
    sizes = [r.RowGroupByteSize(i) for i in range(r.RowGroupCount())]
    rg0, rg1 = pqgpu.plan_row_group_shards(sizes, world)[rank]
    b = r.batch(rg0, rg1, [leaf])
    b.decode()
    shard = pqgather.shard_tensors(b, 0, torch.device("cuda", rank))
    b.close()
    if mode == "all":
        col = pqgather.allgather_column(shard)  # device tensors through RCCL
    else:  # all-to-one on the last rank, point-to-point over RCCL
        col = pqgather.gather_column_to(shard, world - 1)
        if rank != world - 1:
            assert col is None
            dist.destroy_process_group()
            return
    assert all(v.is_cuda for v in col.values() if hasattr(v, "is_cuda"))
    col = pqgather.to_numpy(col)
    if rank == (0 if mode == "all" else world - 1):
        np.savez(os.path.join(out_dir, "gathered.npz"), **{k: np.asarray(v) for k, v in col.items()})
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.timeout(300)
@pytest.mark.parametrize("name,leaf,mode", [("c4_list_str", 0, "all"), ("c4_list_str", 1, "all"),
                                            ("c3_delta_v2", 1, "all"), ("c4_list_str", 1, "root")])
def test_gpu_allgather_rccl_device_tensors(tmp_path, name, leaf, mode):
    """allgather_column over RCCL on device tensors (one rank per GPU the box
    has: RCCL does not put two ranks on one GPU); the gloo tests above cover
    the re-packing at shard boundaries with more ranks."""
    import torch
    import torch.multiprocessing as mp
    import oracle
    world = torch.cuda.device_count()
    if world < 2:
        pytest.skip("an RCCL all-gather needs >= 2 GPUs (a 1-rank 'collective' proves nothing); "
                    "the gloo tests cover the re-packing")
    path = os.path.join(GOLDEN, name + ".parquet")
    mp.spawn(_gpu_rccl_main, args=(world, _free_port(), path, leaf, str(tmp_path), mode), nprocs=world, join=True)
    got = np.load(str(tmp_path / "gathered.npz"))
    o = oracle.File(open(path, "rb").read())
    whole, info = o.decode(leaf), o.leaves()[leaf]
    assert int(got["slots"]) == whole["slots"]
    for k in ("values", "validity", "list_offsets", "list_validity", "str_offsets"):
        if k == "validity" and info["max_def"] == 0:
            continue
        assert np.array_equal(got[k].view(np.uint8).ravel(), whole[k]), k
