"""Chunk -> data node / GPU partitioning and chunk storage keys.

Restated from the reference (pinned by tests/golden/selection_cases.json):
  getIdHash / getObjPartition   hsds/util/idUtil.py:61-66, 481-486  (md5 prefix modulo count)
  getS3Key for chunk ids        hsds/util/idUtil.py:174-251          (schema v2 keys)
With `count` = number of GPUs, getObjPartition is the multi-GPU sharding rule
(SURVEY.md section 8e): identical to HSDS's chunk -> DN rule when dn_count == count.
"""
import functools
import hashlib


def getIdHash(obj_id):
    return hashlib.md5(obj_id.encode("utf8")).hexdigest()[:5]


def getObjPartition(obj_id, count):
    return int(getIdHash(obj_id), 16) % count


def _hex32(obj_id):
    """The 32 hex characters of a v2 id (after the 'x-' / 'cN-' prefix), no dashes."""
    n = obj_id.find("-")
    uuid = obj_id[n + 1:]
    if "_" in uuid:
        uuid = uuid[:uuid.index("_")]
    return uuid.replace("-", "")


@functools.lru_cache(maxsize=1 << 18)
def getS3Key(chunk_id):
    """Storage key of an HSDS v2 chunk id: db/<8>-<8>/d/<4>-<6>-<6>[/p<N>]/<i>_<j>...
    (memoised: a DN computes the keys of the same chunks request after request)"""
    if not chunk_id.startswith("c"):
        raise ValueError(f"Unexpected id: {chunk_id}")
    h = _hex32(chunk_id)
    key = f"db/{h[0:8]}-{h[8:16]}/d/{h[16:20]}-{h[20:26]}-{h[26:32]}"
    n = chunk_id.find("-")
    if n > 1:
        key += "/p" + chunk_id[1:n]
    return key + "/" + chunk_id[chunk_id.index("_") + 1:]


def shard_chunks(chunk_ids, count):
    """{gpu: [chunk ids]} using the reference partition rule."""
    out = {g: [] for g in range(count)}
    for cid in chunk_ids:
        out[getObjPartition(cid, count)].append(cid)
    return out
