"""Row-group sharding across the GPUs of one node (north_star: "Row groups are
independent, so they are sharded round-robin across the 8 GPUs of one node").

One process per GPU: rank r decodes row groups r, r + N, r + 2N, ... on its own context and
stream and returns the decoded columns to the host. There is no collective on the data path;
`reassemble` restores file order (ParquetReader delivers rows ORDERED, ParquetReader.java:225-227)
from the per-rank results wherever they are gathered. torch.distributed is only used by callers
for barriers and timing (bench.py)."""


def row_groups_for_rank(num_row_groups, rank, world):
    """Round-robin: row group g belongs to rank g % world."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of {world}")
    return list(range(rank, num_row_groups, world))


def owner(row_group, world):
    return row_group % world


def reassemble(per_rank, num_row_groups):
    """per_rank[r] = {row_group: result} for the row groups rank r owns -> results in file order.
    Raises if a row group is missing or decoded twice."""
    out = [None] * num_row_groups
    for r, res in enumerate(per_rank):
        for g, v in res.items():
            if owner(g, len(per_rank)) != r:
                raise ValueError(f"row group {g} decoded by rank {r}, owner is {owner(g, len(per_rank))}")
            if out[g] is not None:
                raise ValueError(f"row group {g} decoded twice")
            out[g] = v
    missing = [g for g, v in enumerate(out) if v is None]
    if missing:
        raise ValueError(f"row groups not decoded: {missing}")
    return out


def balance(num_row_groups, world):
    """Max / mean row groups per rank (device-resident scaling efficiency bound)."""
    counts = [len(row_groups_for_rank(num_row_groups, r, world)) for r in range(world)]
    mean = num_row_groups / world
    return max(counts) / mean if mean else 1.0
