"""Multi-process tests of the distributed layer (qe_hip/distributed.py):
gloo on the CPU (world_size 2 and 4) for the exchange plumbing, and a two-rank
rehearsal on one GPU (both ranks compute on cuda:0, collectives over gloo)
for shuffle join, partial/final group-by and the broadcast metric pipeline."""
import os
import socket
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch(mode, world, timeout=300):
    port = free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   LOCAL_RANK="0")
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "dist_worker.py"), mode], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append((p.returncode, out.decode(errors="replace")))
    for rc, out in outs:
        assert rc == 0, out[-3000:]


@pytest.mark.parametrize("world", [2, 4])
def test_exchange_gloo_cpu(world):
    launch("exchange", world)


@pytest.mark.parametrize("world", [2, 3])
def test_exchange_variable_size_payloads_gloo_cpu(world):
    launch("exchange_bytes", world)


@pytest.mark.parametrize("world", [2, 3])
def test_exchange_chunked_rounds_gloo_cpu(world):
    """The round / chunk / local-copy logic of the exchange (shared with the RCCL branch) with a
    40-byte chunk: many rounds, uneven and zero partitions, a rank with no rows."""
    launch("exchange_chunked", world)


def test_a2a_round_plan_pairs_up():
    """_a2a_rounds over random job-wide split matrices: every rank plans the same number of
    rounds, in every round what rank i sends to rank j is exactly what j expects from i, and the
    slices tile each remote partition once, in order."""
    import numpy as np
    from qe_hip.distributed import _a2a_rounds, _peak_remote
    r = np.random.default_rng(5)
    for _ in range(200):
        world = int(r.integers(2, 6))
        S = r.integers(0, 50, (world, world)) * (r.random((world, world)) > 0.3)
        chunk, row_bytes = int(r.integers(1, 200)), int(r.choice([1, 4, 8, 24]))
        peak = _peak_remote(S)
        plans = [_a2a_rounds(list(S[i]), list(S[:, i]), i, row_bytes, chunk, peak) for i in range(world)]
        assert len({len(p) for p in plans}) == 1
        for i in range(world):
            for j in range(world):
                if i == j:
                    assert all(rd[j] == (0, 0, 0, 0) for rd in plans[i])
                    continue
                sent = [(rd[j][0], rd[j][1]) for rd in plans[i]]
                got = [(rd[i][2], rd[i][3]) for rd in plans[j]]
                assert sent == got
                pos = 0
                for a, b in sent:
                    assert a == pos or a == b
                    pos = max(pos, b)
                assert pos == S[i][j]


@pytest.mark.gpu
def test_device_exchange_two_ranks_on_one_gpu():
    """§8 f2: DistributedExecutor.exchange with the device Partitioner (Hash / Range / Single) over
    Int64, Float64, Utf8 and Boolean columns with NULLs; rows conserved, equal keys share a rank,
    range ownership exact."""
    launch("gpu_exchange", 2, timeout=600)


def test_partial_final_decomposition():
    """The partial->final mapping of distributed/planner.rs:200-249: COUNT
    partials are summed, SUM/MIN/MAX partials re-aggregate with themselves."""
    import numpy as np
    from qe_hip.distributed import FINAL_OF
    from qe_hip import AggregateFunction as AF
    r = np.random.default_rng(0)
    k = r.integers(0, 20, 10_000)
    v = r.integers(-50, 50, 10_000)
    shards = np.array_split(np.arange(10_000), 3)
    for f, npf in [(AF.Sum, np.sum), (AF.Count, len), (AF.Min, np.min), (AF.Max, np.max)]:
        final = {}
        for s in shards:
            for key in np.unique(k[s]):
                part = npf(v[s][k[s] == key])
                fin = FINAL_OF[f]
                comb = {AF.Sum: lambda a, b: a + b, AF.Min: min, AF.Max: max}[fin]
                final[key] = comb(final[key], part) if key in final else part
        for key in np.unique(k):
            assert final[key] == npf(v[k == key])


@pytest.mark.gpu
def test_two_ranks_on_one_gpu():
    launch("gpu", 2, timeout=600)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3, 8])
def test_device_tensor_collectives_several_ranks_on_one_gpu(world):
    """The RCCL path's device-tensor code at world size 2, 3 and 8 (collectives over gloo on CUDA
    tensors, ranks sharing one GPU; 8 = one node's ranks, so config 4's 8-way round plan and HIP legs
    run with eight ranks): config 4's shuffle join and the sharded broadcast join with the
    overlapped all-gather + adopted prelaunch and the dense final aggregate, vs the oracle; a build
    key on two ranks (the table form's check clears the summed entry, every rank falls back); probe
    keys crowded into one slice (every rank takes the overflow redo); validity agreed across ranks;
    the chunked all-to-all in many rounds."""
    launch("gpu_devtensors", world, timeout=900)


@pytest.mark.gpu
def test_rccl_world_size_one():
    """The "nccl" backend (RCCL) with world_size 1 on the GPU: exchange, shuffle join,
    partial/final GROUP BY, the sharded broadcast join and config 4's shuffle join vs the oracle."""
    launch("nccl1", 1, timeout=300)


@pytest.mark.gpu
def test_config4_shuffle_join_two_ranks_on_one_gpu():
    """BASELINE config 4 (hash-partitioned join + aggregate) and the sharded broadcast join over two
    ranks (gloo, one GPU) vs the oracle; an exchange where only one shard carries NULLs."""
    launch("gpu_cfg4", 2, timeout=300)


@pytest.mark.gpu
def test_device_tensor_round_trip(ctx):
    """The RCCL path's column <-> cuda-tensor conversion (device copies and
    validity bytes), exercised in one process without a collective."""
    import numpy as np
    import torch
    import torch.distributed as dist
    from qe_hip.distributed import DistributedExecutor
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{free_port()}", rank=0, world_size=1)
    try:
        dx = DistributedExecutor(ctx)
        dx.device = "cuda"
        torch.cuda.set_stream(torch.cuda.Stream())
        ctx.set_stream(torch.cuda.current_stream().cuda_stream)
        r = np.random.default_rng(1)
        for vals in [r.integers(-5, 5, 10_001).astype(np.int64), r.random(777), r.integers(0, 9, 65).astype(np.int32)]:
            m = r.random(len(vals)) > 0.3
            src = ctx.upload(vals, m, offset=3)
            ts = dx._to_tensors(src)
            ctx.sync()
            back = dx._from_tensors(src.dtype, ts[0], ts[1])
            bv, bm = back.to_numpy()
            assert np.array_equal(bm, m) and np.array_equal(bv[m], vals[m])
        ctx.set_stream(0)
    finally:
        dist.destroy_process_group()
