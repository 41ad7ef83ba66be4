"""Optional column materialisation across GPUs.

Decoding needs no collective: row groups are independent (one dictionary per
chunk, chunk_reader.go:221-251) and each rank decodes its own shard.  This
module is the one exchange step §8(e) allows: an all-gather that gives every
rank the whole column, assembled in row-group order from the ranks' shards.

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


def allgather_column(shard, group=None):
    """Whole column on every rank from each rank's decoded shard (row groups in
    rank order, as pqgpu.plan_row_group_shards assigns them).

    shard: dict as returned by shard_tensors (or the same keys as host/CPU
    tensors for gloo): values uint8, validity uint8 bitmap or None,
    list_offsets int32 or None, list_validity uint8 or None, str_offsets
    int64 or None, plus slots / rows ints.
    Returns the same keys for the whole column.
    """
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
        raise ValueError("allgather_column: ranks hold different column layouts")
    slots = [m[0] for m in metas]
    rows = [m[1] for m in metas]
    vbytes = [m[2] for m in metas]
    out = {"slots": sum(slots), "rows": sum(rows), "value_width": shard.get("value_width", 0)}
    out["values"] = torch.cat(_gather_v(shard["values"], vbytes, group))
    if has[0]:
        parts = _gather_v(shard["validity"], [(s + 7) // 8 for s in slots], group)
        out["validity"] = _bool_to_bits(torch.cat([_bits_to_bool(p, s) for p, s in zip(parts, slots)]))
    else:
        out["validity"] = None
    if has[1]:
        # list offsets index element slots: rank r's offsets shift by the
        # element slots of ranks < r
        parts = _gather_v(shard["list_offsets"], [r + 1 for r in rows], group)
        base, segs = 0, [torch.zeros(1, dtype=torch.int32, device=dev)]
        for p, s in zip(parts, slots):
            segs.append(p[1:] - p[0] + base)
            base += s
        out["list_offsets"] = torch.cat(segs)
    else:
        out["list_offsets"] = None
    if has[2]:
        parts = _gather_v(shard["list_validity"], [(r + 7) // 8 for r in rows], group)
        out["list_validity"] = _bool_to_bits(torch.cat([_bits_to_bool(p, r) for p, r in zip(parts, rows)]))
    else:
        out["list_validity"] = None
    if has[3]:
        # string offsets: one per slot + 1, rebased by the preceding shards' bytes
        parts = _gather_v(shard["str_offsets"], [s + 1 for s in slots], group)
        base, segs = 0, [torch.zeros(1, dtype=torch.int64, device=dev)]
        for p, nb in zip(parts, vbytes):
            segs.append(p[1:] - p[0] + base)
            base += nb
        out["str_offsets"] = torch.cat(segs)
    else:
        out["str_offsets"] = None
    return out


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
