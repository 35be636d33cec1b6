"""One-shot IPC all-reduce (csrc/kernels/allreduce.hip) with W processes on the test box's GPU:
bitwise equal to an fp32 rank-ordered sum, across repeated calls of changing sizes (epoch parity)
and inside a captured HIP graph replayed with new contents.  The ranks share one device here (the
box has one GPU); across GPUs the same code reads peers over xGMI."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_tensor(rank, n, salt):
    g = torch.Generator().manual_seed(1000 * salt + rank)
    return torch.randn(n, generator=g).to(torch.bfloat16)


def _expected(world, n, salt):
    acc = _rank_tensor(0, n, salt).float()
    for r in range(1, world):
        acc = acc + _rank_tensor(r, n, salt).float()
    return acc.to(torch.bfloat16)


def _body(rank, world, port, out_dir, uncached=True):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from django_assistant_bot_amd.parallel.custom_allreduce import CustomAllReduce

    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ar = CustomAllReduce(None, dev, max_bytes=4 << 20, spin_limit=1 << 22, uncached=uncached)
    errors = []
    try:
        sizes = [8, 64, 4096 + 8, 1 << 16, (4 << 20) // 2, 3000 * 8, 8]  # elements (x2 bytes)
        for salt, n in enumerate(sizes * 2):  # every size twice: both staging halves
            x = _rank_tensor(rank, n, salt).to(dev)
            ar.all_reduce(x)
            torch.cuda.synchronize()
            if not torch.equal(x.cpu(), _expected(world, n, salt)):
                errors.append(f"eager n={n} salt={salt}")
        ar.check_error()
        # graph capture: 3 all-reduces of a static buffer, replayed with new inputs
        n = 4096 * 8
        buf = torch.zeros(n, dtype=torch.bfloat16, device=dev)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            ar.all_reduce(buf)  # warm-up outside the graph (keeps the epochs in step on every rank)
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            ar.all_reduce(buf)
            buf.mul_(0.5)
            ar.all_reduce(buf)
        for it in range(5):
            salt = 100 + it
            buf.copy_(_rank_tensor(rank, n, salt).to(dev))
            torch.cuda.synchronize()
            dist.barrier()
            g.replay()
            torch.cuda.synchronize()
            once = (_expected(world, n, salt).float() * 0.5).to(torch.bfloat16)
            exp = once.float() * world  # every rank holds `once` before the second reduce
            exp = exp.to(torch.bfloat16)
            if not torch.allclose(buf.cpu().float(), exp.float(), rtol=1e-2, atol=1e-2):
                errors.append(f"graph replay {it}")
        ar.check_error()
        # fused slab sum + all-reduce + residual + RMSNorm: bitwise the unfused sequence
        from django_assistant_bot_amd import ops

        for rows, cols, S in ((3, 4096, 8), (128, 8192, 4), (70, 1024, 1), (128, 4096, 0)):
            def part(r):
                g = torch.Generator().manual_seed(7000 + 31 * r + rows)
                if S == 0:
                    return torch.randn(rows, cols, generator=g).to(torch.bfloat16).to(dev)
                return torch.randn(S, rows, cols, generator=g).to(dev)
            g = torch.Generator().manual_seed(99 + rows)
            res = torch.randn(rows, cols, generator=g).to(torch.bfloat16).to(dev)
            w = (0.5 + torch.rand(cols, generator=g)).to(torch.bfloat16).to(dev)
            out, res_out = ar.all_reduce_rmsnorm(part(rank), res, w, 1e-5)
            torch.cuda.synchronize()
            acc = None
            for r in range(world):
                p_r = part(r)
                p_r = ops.slab_reduce(p_r) if S else p_r
                acc = p_r.float() if acc is None else acc + p_r.float()
            exp_out, exp_res = ops.rmsnorm(acc.to(torch.bfloat16), w, 1e-5, residual=res)
            if not (torch.equal(out, exp_out) and torch.equal(res_out, exp_res)):
                errors.append(f"fused norm rows={rows} cols={cols} S={S}")
        ar.check_error()
    except Exception as exc:  # report, do not hang the other ranks' joins
        errors.append(repr(exc))
    finally:
        ar.close()
        with open(os.path.join(out_dir, f"r{rank}.txt"), "w") as f:
            f.write("\n".join(errors) if errors else "ok")
        dist.destroy_process_group()


@pytest.mark.parametrize("world,uncached", [(2, True), (4, True), (8, True), (2, False)])
def test_one_shot_allreduce_multi_process(world, uncached, tmp_path):
    """world 8 = the TP-8 group of a 70B node (here 8 processes on one device)."""
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_body, args=(r, world, port, str(tmp_path), uncached)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    alive = [p for p in procs if p.is_alive()]
    for p in alive:
        p.kill()
    assert not alive, "all-reduce ranks hung"
    res = [open(tmp_path / f"r{r}.txt").read() for r in range(world)]
    assert res == ["ok"] * world, res


@pytest.mark.parametrize("rows,cols,S", [(1, 8192, 8), (7, 4096, 4), (128, 4096, 8), (128, 8192, 2), (200, 1024, 0)])
def test_fused_allreduce_rmsnorm_is_the_unfused_sequence_at_tp1(rows, cols, S):
    """one launch (slab sum -> one-shot all-reduce -> residual -> RMSNorm) is
    bit-identical to slab_reduce + all_reduce + rmsnorm, here at W = 1 (one process)."""
    from django_assistant_bot_amd import ops
    from django_assistant_bot_amd.parallel.custom_allreduce import CustomAllReduce

    dev = torch.device("cuda", 0)
    ar = CustomAllReduce(None, dev, max_bytes=4 << 20)
    try:
        g = torch.Generator().manual_seed(rows * 7 + S)
        part = (torch.randn(S, rows, cols, generator=g).to(dev) if S else
                torch.randn(rows, cols, generator=g).to(torch.bfloat16).to(dev))
        res = torch.randn(rows, cols, generator=g).to(torch.bfloat16).to(dev)
        w = (0.5 + torch.rand(cols, generator=g)).to(torch.bfloat16).to(dev)
        out, res_out = ar.all_reduce_rmsnorm(part, res, w, 1e-5)
        x = ops.slab_reduce(part) if S else part.clone()
        ar.all_reduce(x)
        exp_out, exp_res = ops.rmsnorm(x, w, 1e-5, residual=res)
        torch.cuda.synchronize()
        assert torch.equal(out, exp_out) and torch.equal(res_out, exp_res)
        ar.check_error()
    finally:
        ar.close()
