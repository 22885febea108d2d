"""The tensor-parallel FUSED decode step (``forward_decode_fused_tp``: the residual updated in place by the all-reduce,
``TPInfo.row_parallel`` for o / down, vocab-parallel lm_head + gather) on CPU reference ops over
gloo, against the unsharded tp=1 fused step with the same ``random-full`` weights.

On a GPU group ``row_parallel`` may run the fused GEMM + one-shot all-reduce (csrc/oneshot_ar.hip);
on CPU it is the reference GEMM + gloo all-reduce, so this pins the data flow of the TP step (which
buffer holds the residual after each NORM_ADD, what each rank's shard contributes) independently
of the kernels. The GPU twin is tests/test_distributed_gpu.py::test_tp_fused_decode_matches_tp1_on_shared_gpu."""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from test_distributed_cpu import free_port


def _decode_step(e, prompt: str):
    from theroundtaible_amd.models.llama import AttnMeta
    ids = e.encode_prompt(prompt)
    s = e.kv.seq("probe")
    pre = e.prefill([(s, ids)])
    e.kv.ensure_capacity(s, s.length + 1)
    p = s.length
    pos = torch.tensor([p])
    slots = torch.tensor([s.blocks[p // e.kv.block_size] * e.kv.block_size + p % e.kv.block_size])
    bt = torch.tensor([s.blocks], dtype=torch.int32)
    meta = AttnMeta("decode", slots, bt, (pos + 1).to(torch.int32), num_splits=1)
    nxt = torch.tensor([int(pre[0].argmax())])
    if e.tp.size > 1:
        return e.model.forward_decode_fused_tp(nxt, pos, e.kv, meta)
    return e.model.forward_decode_fused(nxt, pos, e.kv, meta)


def _engine(tp=None):
    from theroundtaible_amd.engine import Engine, EngineConfig
    return Engine(EngineConfig(model="tiny-llama", device="cpu", dtype="fp32", num_blocks=64,
                               weights="random-full:11"), tp)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from theroundtaible_amd.parallel.tp import TPInfo
        tp = TPInfo(size=world, rank=rank, group=dist.group.WORLD)
        e = _engine(tp)
        logits = _decode_step(e, "de gedeelde ronde tafel")
        if rank == 0:
            q.put(logits.tolist())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_tp_fused_decode_step_matches_tp1_on_cpu(world):
    ref = _decode_step(_engine(), "de gedeelde ronde tafel")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    logits = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    got = torch.tensor(logits)
    assert got.shape == ref.shape
    assert torch.allclose(got, ref, atol=2e-3, rtol=2e-3), (got - ref).abs().max()
