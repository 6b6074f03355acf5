"""DN micro-batcher: concurrent chunk requests coalesced into one engine batch.

The reference decodes one chunk per HTTP request: GET_Chunk (hsds/chunk_dn.py:317) calls
get_chunk (hsds/datanode_lib.py:948) and chunkReadSelection (hsds/util/chunkUtil.py:882)
for its one chunk, and the SN crawler keeps up to max_tasks_per_node_per_request (16) x
dn_count such requests in flight (hsds/chunk_crawl.py:629-663); concurrent reads of one
chunk id wait on the first (pending_s3_read, datanode_lib.py:1041-1065).  One stream per
request is 1-4 zlib streams on a GPU that needs thousands to be busy, so the DN side
gathers the requests that arrive within a short window (or up to max_batch of them) into
ONE ChunkStore.get_chunks batch -- one decode launch -- and ONE selection-gather launch
with one device-to-host copy for all their chunkReadSelection results.  Requests for the
same chunk id in a window share one read (the reference's dedupe); requests whose dataset
parameters differ (dtype, layout, filters, fill value) form separate groups.

The engine is re-entrant (include/hsds_amd.h, "Threading"), so batches run on a worker
thread off the event loop, as the reference's blosc_nthreads codec work would.
"""
import asyncio
import json
from concurrent.futures import ThreadPoolExecutor

import numpy as np

__all__ = ["ChunkBatcher"]


def _freeze(x):
    try:
        return json.dumps(x, sort_keys=True, default=str)
    except TypeError:
        return repr(x)


class ChunkBatcher:
    """Coalesces `get_selection` / `get_chunk` coroutine calls into batches.

    `store` is a hsds_amd.datanode.ChunkStore (or anything with its get_chunks
    signature).  window_ms: how long the first request of a batch waits for company;
    max_batch: a full batch is dispatched at once.  stats["batches"] counts the
    get_chunks calls, stats["requests"] the requests served, stats["reads"] the distinct
    chunk reads issued."""

    def __init__(self, store, window_ms=0.5, max_batch=4096, executor=None):
        self.store = store
        self.window = window_ms / 1e3
        self.max_batch = max_batch
        self.executor = executor or ThreadPoolExecutor(max_workers=1, thread_name_prefix="hsds-amd-batch")
        self._groups = {}        # group key -> {"reqs": [...], "timer": handle}
        self.stats = {"batches": 0, "requests": 0, "reads": 0}

    async def get_selection(self, read, dtype, chunk_dims, slices=None, filter_ops=None, fill_value=None,
                            layout_class=None, hyper_dims=None, chunk_init=False):
        """chunkReadSelection(get_chunk(...), slices) as a host ndarray (GET_Chunk's
        response array, chunk_dn.py:552); None when the chunk does not exist (404) and
        chunk_init is off; a read error raises as get_chunk would."""
        loop = asyncio.get_running_loop()
        dtype = np.dtype(dtype)
        chunk_dims = tuple(int(c) for c in chunk_dims)
        key = (dtype.str, chunk_dims, _freeze(filter_ops), _freeze(fill_value), layout_class,
               None if hyper_dims is None else tuple(hyper_dims), bool(chunk_init))
        g = self._groups.get(key)
        if g is None:
            g = {"reqs": [], "timer": None, "args": (dtype, chunk_dims, filter_ops, fill_value, layout_class,
                                                     hyper_dims, chunk_init)}
            self._groups[key] = g
            g["timer"] = loop.call_later(self.window, self._dispatch, key)
        fut = loop.create_future()
        g["reqs"].append((read, None if slices is None else tuple(slices), fut))
        if len(g["reqs"]) >= self.max_batch:
            g["timer"].cancel()
            self._dispatch(key)
        return await fut

    async def get_chunk(self, read, dtype, chunk_dims, **kw):
        """get_chunk as a host ndarray of the full chunk (or None for a 404)."""
        return await self.get_selection(read, dtype, chunk_dims, None, **kw)

    def _dispatch(self, key):
        g = self._groups.pop(key, None)
        if g is None or not g["reqs"]:
            return
        loop = asyncio.get_running_loop()
        reqs = g["reqs"]
        task = loop.run_in_executor(self.executor, self._run_batch, reqs, g["args"])
        task.add_done_callback(lambda t, reqs=reqs: self._finish(t, reqs))

    def _finish(self, task, reqs):
        exc = task.exception()
        if exc is not None:
            for _, _, fut in reqs:
                if not fut.done():
                    fut.set_exception(exc)
            return
        for (_, _, fut), res in zip(reqs, task.result()):
            if fut.done():
                continue
            if isinstance(res, BaseException):
                fut.set_exception(res)
            else:
                fut.set_result(res)

    def _run_batch(self, reqs, args):
        dtype, chunk_dims, filter_ops, fill_value, layout_class, hyper_dims, chunk_init = args
        # one read per distinct chunk id (the reference's in-flight dedupe)
        order, index = [], {}
        for read, _, _ in reqs:
            if read.chunk_id not in index:
                index[read.chunk_id] = len(order)
                order.append(read)
        vals = self.store.get_chunks(order, dtype, chunk_dims, filter_ops=filter_ops, fill_value=fill_value,
                                     layout_class=layout_class, hyper_dims=hyper_dims, chunk_init=chunk_init)
        self.stats["batches"] += 1
        self.stats["reads"] += len(order)
        self.stats["requests"] += len(reqs)
        items = []
        for read, slices, _ in reqs:
            v = vals[index[read.chunk_id]]
            items.append((v, slices))
        return _gather(self.store, items, dtype, chunk_dims)


def _gather(store, items, dtype, chunk_dims):
    """The selections of one batch: device chunks through ONE copy launch into a packed
    device buffer and ONE device-to-host copy; host arrays (a CPU store) by numpy."""
    out = [None] * len(items)
    dev_items = []
    for k, (v, slices) in enumerate(items):
        if v is None or isinstance(v, BaseException):
            out[k] = v
        elif isinstance(v, np.ndarray):
            a = v.reshape(chunk_dims) if v.dtype == dtype else v.view(dtype).reshape(chunk_dims)
            out[k] = np.ascontiguousarray(a if slices is None else a[slices])
        else:
            dev_items.append(k)
    if dev_items:
        import torch
        from .engine import ChunkEngine
        from .selection import copy_desc, _contig_slices
        abase = store.cache.arena.buf
        full = tuple(slice(0, n, 1) for n in chunk_dims)
        recs, shapes, offs, total = [], [], [], 0
        for k in dev_items:
            v, slices = items[k]
            sl = full if slices is None else slices
            shape = tuple(len(range(*s.indices(n))) for s, n in zip(sl, chunk_dims))
            nbytes = int(np.prod(shape, dtype=np.int64)) * dtype.itemsize
            shapes.append(shape)
            offs.append(total)
            if nbytes:
                recs.append(copy_desc(chunk_dims, sl, shape, _contig_slices(shape), dtype.itemsize,
                                      src_base=v.data_ptr() - abase.data_ptr(), dst_base=total))
            total += (nbytes + 255) // 256 * 256
        packed = torch.empty(max(total, 1), dtype=torch.uint8, device=abase.device)
        if recs:
            ChunkEngine(abase.device.index).copy(abase, packed, np.concatenate(recs))
        host = packed.cpu().numpy()
        for k, shape, o in zip(dev_items, shapes, offs):
            n = int(np.prod(shape, dtype=np.int64)) * dtype.itemsize
            out[k] = host[o:o + n].view(dtype).reshape(shape).copy()
    return out
