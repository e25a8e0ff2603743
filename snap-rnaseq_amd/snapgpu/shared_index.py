"""Build the seed index once per node and share it with every rank.

The reference is one process: one GenomeIndex in one address space.  A multi-GPU job here is
one process per GPU; instead of every rank generating the genome and building its own index
(for GRCh38 that is 8 concurrent builds of tens of GB), local rank 0 of each node builds it,
writes the flat shared form (snapgpu_index_share) under the node's /dev/shm, and every other
rank of that node maps it read-only (snapgpu_index_attach) and uploads the tables to its own
GPU's HBM.  gloo carries only the barrier; the index bytes never go through a collective.
"""
import os
import time

SHM_DIR = "/dev/shm"


def _path(tag):
    port = os.environ.get("MASTER_PORT", "0")
    return os.path.join(SHM_DIR, f"snapgpu_index_{port}_{tag}.bin")


def _node_local():
    """(local rank, ranks on this node) from torch.distributed.run's environment."""
    return int(os.environ.get("LOCAL_RANK", "0")), int(os.environ.get("LOCAL_WORLD_SIZE", "0"))


def build_once(snapgpu, genome_bases, gen, seed_len, n_threads, rank, world, dist):
    """-> (GenomeIndex, info dict).  gen: Genome.synthetic keyword arguments.  One build per
    node: the builder is LOCAL_RANK 0 (global rank 0 when the launcher sets no LOCAL_RANK)."""
    tag = f"{genome_bases}_{gen.get('seed', 0)}_{gen.get('n_contigs', 1)}_{gen.get('n_repeat_families', 0)}_{seed_len}"
    local, local_world = _node_local()
    builder = (local == 0) if "LOCAL_RANK" in os.environ else (rank == 0)
    share = world > 1 and (local_world == 0 or local_world > 1)
    info = {"ranks": world}
    if builder:
        t0 = time.time()
        g = snapgpu.Genome.synthetic(genome_bases, **gen)
        info["genome_s"] = round(time.time() - t0, 2)
        t1 = time.time()
        idx = snapgpu.GenomeIndex.build(g, seed_len, n_threads)
        info["build_s"] = round(time.time() - t1, 2)
        info["built_by_this_rank"] = True
        ii = idx.info()
        info.update(slots=ii["totalHashSlots"], used_slots=ii["totalUsedSlots"],
                    overflow_words=ii["overflowTableSize"], load_factor=round(ii["totalUsedSlots"] / ii["totalHashSlots"], 4))
        if share:
            t2 = time.time()
            idx.share(_path(tag))
            info["share_s"] = round(time.time() - t2, 2)
            info["shared_file"] = _path(tag)
            # one image per node in host RAM: the builder drops its private index and maps the shared
            # file like every other rank (C3: 56 GB once, not once per rank plus the file)
            del idx, g
            idx = snapgpu.GenomeIndex.attach(_path(tag))
            info["attached"] = True
    if dist is not None:
        dist.barrier()
    if not builder:
        t3 = time.time()
        idx = snapgpu.GenomeIndex.attach(_path(tag))
        info["attach_s"] = round(time.time() - t3, 3)
        info["built_by_this_rank"] = False
        info["shared_file"] = _path(tag)
        info["attached"] = True
    return idx, info


def cleanup(rank, world):
    """The node's builder removes its shared file once every rank has attached (mappings stay
    valid); call after a barrier."""
    local, _ = _node_local()
    builder = (local == 0) if "LOCAL_RANK" in os.environ else (rank == 0)
    if not builder or world <= 1:
        return
    for f in os.listdir(SHM_DIR):
        if f.startswith(f"snapgpu_index_{os.environ.get('MASTER_PORT', '0')}_"):
            try:
                os.unlink(os.path.join(SHM_DIR, f))
            except OSError:
                pass
