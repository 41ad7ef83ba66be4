"""Optional column materialisation across GPUs.

Decoding needs no collective: row groups are independent (one dictionary per
chunk, chunk_reader.go:221-251) and each rank decodes its own shard.  This
module is the one exchange step §8(e) allows, in two forms: `gather_column_to`
materialises the whole column on one device (all-to-one point-to-point sends,
the topology SURVEY.md §5 prefers over xGMI), `allgather_column` gives every
rank the whole column; both assemble it in row-group order from the shards.

* fixed-width values, validity bitmaps, list validity: all-gather-v (shards
  padded to the largest, one `all_gather` per buffer, then trimmed);
* bitmaps are re-packed at the shard boundaries (a shard's slot count is not a
  multiple of 8 in general);
* string offsets (int64) and list offsets (int32) are rebased by the preceding
  shards' byte / element counts, the way `ColumnStore` concatenates pages
  (data_store.go:15-31).

The collective is whatever `torch.distributed` was initialised with: RCCL over
xGMI for device tensors ("nccl"), gloo for the CPU tests.  It is never part of
the decode timing: `bench.py --gpus N --allgather` times it separately after
the timed steps and reports it as `config.allgather`.
"""
import ctypes

import numpy as np

import pqgpu

_HIP = None


def _hip():
    global _HIP
    if _HIP is None:
        _HIP = ctypes.CDLL("libamdhip64.so")
        _HIP.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    return _HIP


def shard_tensors(batch, i, device):
    """Device copies (torch tensors on `device`) of selected column i of a
    decoded batch: the inputs of `allgather_column`.  The copy is device to
    device (hipMemcpyDeviceToDevice), so the shard never leaves HBM."""
    import torch
    batch.sync()
    v = batch.view(i)
    out = {"slots": int(v.slots), "rows": int(v.rows), "value_width": int(v.value_width)}
    for name, buf, ptr, dt in (("values", pqgpu.BUF_VALUES, v.values, torch.uint8),
                               ("validity", pqgpu.BUF_VALIDITY, v.validity, torch.uint8),
                               ("list_offsets", pqgpu.BUF_LIST_OFFSETS, v.list_offsets, torch.int32),
                               ("list_validity", pqgpu.BUF_LIST_VALIDITY, v.list_validity, torch.uint8),
                               ("str_offsets", pqgpu.BUF_STR_OFFSETS, v.str_offsets, torch.int64)):
        # a buffer exists when the column's schema has it (the view pointer),
        # even when this shard holds no rows of it (an empty shard)
        if not ptr:
            out[name] = None
            continue
        n = ctypes.c_size_t()
        pqgpu._check(pqgpu.lib().pqg_batch_copy(batch._h, i, buf, None, 0, ctypes.byref(n)))
        isz = torch.empty(0, dtype=dt).element_size()
        t = torch.empty(n.value // isz, dtype=dt, device=device)
        if n.value:
            torch.cuda.synchronize(device)
            rc = _hip().hipMemcpy(t.data_ptr(), ptr, n.value, 3)  # hipMemcpyDeviceToDevice
            if rc != 0:
                raise RuntimeError("hipMemcpy device-to-device failed: %d" % rc)
        out[name] = t
    return out


def _gather_v(t, counts, group):
    """all-gather-v of a 1-D tensor: every rank's `t[:counts[r]]`, as a list."""
    import torch
    import torch.distributed as dist
    world = len(counts)
    m = max(counts)
    pad = torch.zeros(m, dtype=t.dtype, device=t.device)
    if t.numel():
        pad[:t.numel()] = t
    parts = [torch.empty(m, dtype=t.dtype, device=t.device) for _ in range(world)]
    dist.all_gather(parts, pad, group=group)
    return [p[:c] for p, c in zip(parts, counts)]


def _bits_to_bool(bm, n):
    import torch
    shifts = torch.arange(8, dtype=torch.uint8, device=bm.device)
    return ((bm.unsqueeze(1) >> shifts) & 1).reshape(-1)[:n].bool()


def _bool_to_bits(b):
    import torch
    n = b.numel()
    pad = torch.zeros((n + 7) // 8 * 8, dtype=torch.uint8, device=b.device)
    pad[:n] = b.to(torch.uint8)
    w = (1 << torch.arange(8, dtype=torch.int32, device=b.device)).to(torch.uint8)
    return (pad.reshape(-1, 8) * w).sum(1, dtype=torch.int32).to(torch.uint8)


def _layout(shard, group):
    """Every rank's (slots, rows, value bytes) and the buffers the column has
    (a tiny all-gather of 7 int64s, the only collective both exchanges share)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    dev = shard["values"].device
    has = [shard.get(k) is not None for k in ("validity", "list_offsets", "list_validity", "str_offsets")]
    meta = torch.tensor([shard["slots"], shard["rows"], shard["values"].numel()] + [int(h) for h in has],
                        dtype=torch.int64, device=dev)
    metas = [torch.empty_like(meta) for _ in range(world)]
    dist.all_gather(metas, meta, group=group)
    metas = [m.tolist() for m in metas]
    if any(m[3:] != metas[0][3:] for m in metas):
        raise ValueError("pqgather: ranks hold different column layouts")
    return [m[0] for m in metas], [m[1] for m in metas], [m[2] for m in metas], has


def _counts(name, slots, rows, vbytes):
    """Elements of buffer `name` in each rank's shard."""
    return {"values": vbytes,
            "validity": [(s + 7) // 8 for s in slots],
            "list_offsets": [r + 1 for r in rows],
            "list_validity": [(r + 7) // 8 for r in rows],
            "str_offsets": [s + 1 for s in slots]}[name]


_BUFS = ("values", "validity", "list_offsets", "list_validity", "str_offsets")


def _assemble(parts, slots, rows, vbytes, has, value_width, dev):
    """The whole column from the shards' buffers in rank (= row-group) order:
    bitmaps re-packed at shard boundaries, offsets rebased (data_store.go:15-31)."""
    import torch
    out = {"slots": sum(slots), "rows": sum(rows), "value_width": value_width}
    out["values"] = torch.cat(parts["values"])
    out["validity"] = None
    if has[0]:
        out["validity"] = _bool_to_bits(torch.cat([_bits_to_bool(p, s) for p, s in zip(parts["validity"], slots)]))
    out["list_offsets"] = None
    if has[1]:
        # list offsets index element slots: rank r's offsets shift by the
        # element slots of ranks < r
        base, segs = 0, [torch.zeros(1, dtype=torch.int32, device=dev)]
        for p, s in zip(parts["list_offsets"], slots):
            segs.append(p[1:] - p[0] + base)
            base += s
        out["list_offsets"] = torch.cat(segs)
    out["list_validity"] = None
    if has[2]:
        out["list_validity"] = _bool_to_bits(
            torch.cat([_bits_to_bool(p, r) for p, r in zip(parts["list_validity"], rows)]))
    out["str_offsets"] = None
    if has[3]:
        # string offsets: one per slot + 1, rebased by the preceding shards' bytes
        base, segs = 0, [torch.zeros(1, dtype=torch.int64, device=dev)]
        for p, nb in zip(parts["str_offsets"], vbytes):
            segs.append(p[1:] - p[0] + base)
            base += nb
        out["str_offsets"] = torch.cat(segs)
    return out


def _present(name, has):
    return name == "values" or has[_BUFS.index(name) - 1]


def allgather_column(shard, group=None):
    """Whole column on every rank from each rank's decoded shard (row groups in
    rank order, as pqgpu.plan_row_group_shards assigns them).

    shard: dict as returned by shard_tensors (or the same keys as host/CPU
    tensors for gloo): values uint8, validity uint8 bitmap or None,
    list_offsets int32 or None, list_validity uint8 or None, str_offsets
    int64 or None, plus slots / rows ints.
    Returns the same keys for the whole column.
    """
    slots, rows, vbytes, has = _layout(shard, group)
    parts = {}
    for name in _BUFS:
        if _present(name, has):
            parts[name] = _gather_v(shard[name], _counts(name, slots, rows, vbytes), group)
    return _assemble(parts, slots, rows, vbytes, has, shard.get("value_width", 0), shard["values"].device)


def gather_column_to(shard, root=0, group=None):
    """Whole column on ONE rank (`root`, a rank of `group`): the all-to-one
    materialisation of SURVEY.md §5 / §8(e).  Every other rank sends its shard's
    buffers straight to the root (point-to-point sends, posted together with
    `batch_isend_irecv`, so over xGMI each source uses its own link to the
    root); nothing is padded and no rank but the root holds the whole column —
    1/N of `allgather_column`'s memory and link traffic.  Same shard dict as
    `allgather_column`; returns the whole column on the root, None elsewhere.
    """
    import torch
    import torch.distributed as dist
    slots, rows, vbytes, has = _layout(shard, group)
    me = dist.get_rank(group)
    world = len(slots)
    g_root = root if group is None else dist.get_global_rank(group, root)
    dev = shard["values"].device
    ops, parts = [], {}
    for name in _BUFS:
        if not _present(name, has):
            continue
        cnt = _counts(name, slots, rows, vbytes)
        t = shard[name]
        if me != root:
            if cnt[me]:
                ops.append(dist.P2POp(dist.isend, t[:cnt[me]].contiguous(), g_root, group))
            continue
        bufs = []
        for r in range(world):
            if r == root:
                bufs.append(t[:cnt[r]])
                continue
            b = torch.empty(cnt[r], dtype=t.dtype, device=dev)
            if cnt[r]:
                src = r if group is None else dist.get_global_rank(group, r)
                ops.append(dist.P2POp(dist.irecv, b, src, group))
            bufs.append(b)
        parts[name] = bufs
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    if me != root:
        return None
    return _assemble(parts, slots, rows, vbytes, has, shard.get("value_width", 0), dev)


def to_numpy(col):
    """Host copy of an allgather_column result in the canonical (oracle) layout."""
    out = {}
    for k, v in col.items():
        if v is None:
            out[k] = np.zeros(0, np.uint8)
        elif hasattr(v, "cpu"):
            out[k] = v.cpu().numpy().view(np.uint8).ravel() if k != "values" else v.cpu().numpy()
        else:
            out[k] = v
    return out
