"""GPU: the N>1 paths with the HIP engine as the per-rank search.

* gpuhash.dist.distributed_min over 2 gloo ranks that share the one GPU, each rank
  searching its shard with its own gpuhash context, the shards cut by the engine's cost
  model (gpuhash_shard_range), on ranges that cross 1 -> 2 SHA blocks -- against the oracle.
* bench.py's two N-GPU modes, rehearsed on the one GPU: `--inproc 0,0` (one process, two
  shards, one stream each) and torch.distributed.run with 2 ranks (GPUHASH_SHARE_GPU=1);
  their merged result must equal one call over the same range.  And `--gpus N` with N
  above the visible devices must fail loudly instead of measuring one GPU.
"""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
M120 = (b"The quick brown fox jumps over the lazy dog. " * 3)[:120]
# m = 45: 9-digit nonces hash 1 block, 10-digit ones 2 (an extra padding block);
# m = 50: the same change at 4 -> 5 digits
CASES = [(M120[:45], 10**9 - (1 << 22), 10**9 + (1 << 22)),
         (M120[:50], 0, 3_000_000),
         (M120, 9_999_000_000, 10_004_000_000),
         (b"bradfitz", 0, 9999)]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    import gpuhash
    import gpuhash.dist as gd
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = []
    with gpuhash.Engine([0]) as eng:
        for msg, lo, hi in CASES:
            shard = gd.split_range(lo, hi, world, msg_len=len(msg))[rank]
            res = gd.distributed_min(lambda a, b: eng.min(msg, a, b), lo, hi, msg_len=len(msg))
            out.append((shard, res))
    q.put((rank, out))
    dist.destroy_process_group()


def test_distributed_min_with_the_hip_engine(oracle):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=100) for _ in range(world))
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    for i, (msg, lo, hi) in enumerate(CASES):
        want = oracle.min(msg, lo, hi, threads=8)
        (s0, r0), (s1, r1) = res[0][i], res[1][i]
        assert r0 == r1 == want, (msg, lo, hi)
        assert s0[0] == lo and s1[1] == hi and s1[0] == s0[1] + 1  # contiguous cost-balanced shards
    # the cost model moves the m = 45 cut past 10^9: the 2-block shard holds fewer nonces
    (a0, b0), (a1, b1) = res[0][0][0], res[1][0][0]
    assert b0 > 10**9 and (b0 - a0) > 1.2 * (b1 - a1)


def _bench(args, env_extra=None, launcher=None, timeout=100):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.update(env_extra or {})
    cmd = (launcher or [sys.executable]) + [os.path.join(ROOT, "bench.py"), *args]
    return subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=timeout, cwd=ROOT)


def test_bench_inproc_two_shards_on_one_gpu(engine):
    """bench.py's in-process N=2 path rehearsed as two shards on the one GPU, INCLUDING the
    default search leg: config 4's whole [0, 2^40) of 'bradfitz' in one gpuhash_min over
    the two shards, checked by bench.py against the committed CPU golden."""
    r = _bench(["--inproc", "0,0", "--steps", "1", "--warmup", "0", "--no-cpu-baseline"], timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["config"]["parallelism"] == "inproc2"
    assert line["config"]["ranges"] == [[0, (2 << 32) - 1]]
    assert tuple(line["result"]) == engine.min(b"bradfitz", 0, (2 << 32) - 1)
    assert line["roofline"]["kernel"] == "k_scan<J=4,C2=0,EX=0,MODE=0>"
    assert len(line["per_device"]) == 1  # both shards report device ordinal 0
    assert [s["shard"] for s in line["shards"]] == [0, 1] and "device_check" not in line
    s = line["search_2p40"]
    assert s["range"] == [0, (1 << 40) - 1] and s["golden_name"] == "cfg4_bradfitz_2p40"
    assert s["matches_golden"] is True and tuple(s["result"]) == (16555811, 890536971553)
    # the two shards' windows (2 slices of 2^39, each cut over both) tile [0, 2^40), each
    # shard on the stream of the device it names
    import bench
    sh = s["shards"]
    assert [x["shard"] for x in sh] == [0, 1] and [x["slices"] for x in sh] == [2, 2]
    assert bench.tiles(sh, 0, (1 << 40) - 1) and sum(x["nonces"] for x in sh) == 1 << 40
    assert all(x["device"] == 0 and x["stream_device"] == [0] for x in sh)
    # same-run scaling evidence: shard 0's windows again, alone.  Two shards sharing one GPU
    # do not scale, so shard 0 alone takes about half the two-shard time
    sc = s["scaling"]
    assert sc["windows"] == sh[0]["windows"] and 0.3 < sc["scaling_efficiency"] < 0.8, sc
    # the timed step's shard rates are per step, near the kernel rate
    assert all(x["nonces_hashed"] == x["nonces"] for x in line["shards"])  # one step here
    assert all(x["kernel_GHs"] > 5 for x in line["shards"])
    # the timed step's [0, 2^33) is checked against its CPU golden (config 2 at N = 2)
    assert line["matches_golden"] is True and line["result_check"]["golden_names"] == ["cfg2_bradfitz_2gpu"]


def test_bench_gpus_above_visible_fails_loudly():
    import gpuhash
    n = gpuhash.device_count() + 1
    r = _bench(["--gpus", str(n), "--steps", "1", "--warmup", "0", "--no-cpu-baseline"])
    assert r.returncode == 2 and "HIP device(s) are visible" in r.stderr
    assert r.stdout.strip() == ""


def test_bench_torchrun_two_ranks_on_one_gpu(engine):
    import bench
    port = _free_port()
    launcher = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                "--master-addr", "127.0.0.1", "--master-port", str(port)]
    r = _bench(["--gpus", "2", "--steps", "1", "--warmup", "0", "--no-cpu-baseline",
                "--search", "0:4294967295"],
               {"GPUHASH_SHARE_GPU": "1"}, launcher=launcher)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["config"]["parallelism"] == "dp2"
    assert line["config"]["backend"] == "gloo"
    # rank r searched [r*2^32, (r+1)*2^32): the merged result is the whole range's argmin
    assert tuple(line["result"]) == engine.min(b"bradfitz", 0, (2 << 32) - 1)
    # the search leg: each rank its cost-balanced window of config 2's range, gloo merge,
    # checked against the committed golden (5256245051, 1626825724)
    s = line["search_2p40"]
    assert s["golden_name"] == "cfg2_bradfitz_2p32" and s["matches_golden"] is True
    assert [x["shard"] for x in s["shards"]] == [0, 1] and s["devices"] == [0, 0]
    assert s["shards"][1]["windows"][0][0] == s["shards"][0]["windows"][-1][1] + 1
    assert "device_check" not in line
    # rank 0 repeats the search in-process over one context of N entries (here ordinal 0
    # twice; on an 8-GPU node devices 0..7), checked against the same golden
    si = line["search_2p40_inproc"]
    assert si["matches_golden"] is True and si["devices"] == [0, 0]
    assert [x["shard"] for x in si["shards"]] == [0, 1] and bench.tiles(si["shards"], 0, (1 << 32) - 1)
    assert 0.3 < s["scaling"]["scaling_efficiency"] < 0.8  # two ranks share the GPU
    assert line["matches_golden"] is True and line["result_check"]["golden_names"] == ["cfg2_bradfitz_2gpu"]
    # without GPUHASH_SHARE_GPU, two ranks on a 1-GPU box must fail loudly: refused at
    # start, or -- when a *_VISIBLE_DEVICES variable leaves each process one GPU, which
    # bench.py accepts as one GPU per rank -- by the PCI check once both ranks report the
    # same physical GPU (exit 3 after the line)
    import gpuhash
    if gpuhash.device_count() == 1:
        r = _bench(["--gpus", "2", "--steps", "1", "--warmup", "0", "--no-cpu-baseline",
                    "--search", "0:4294967295"], launcher=launcher[:-1] + [str(_free_port())])
        assert r.returncode != 0
        assert "LOCAL_RANK 1" in r.stderr or "share a (host, PCI) device" in r.stderr, r.stderr[-1500:]


def test_bench_default_line_checks_its_step(engine):
    """The headline line at N = 1 (config 2, [0, 2^32)) compares its timed step's result with
    the committed golden and reports per-shard rates per step."""
    r = _bench(["--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--search", "off"])
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["matches_golden"] is True and line["result_check"]["golden_names"] == ["cfg2_bradfitz_2p32"]
    (sh,) = line["shards"]
    assert sh["nonces"] == 1 << 32 and sh["nonces_hashed"] == 2 << 32
    assert sh["kernel_GHs"] == pytest.approx(line["per_device"][0]["kernel_GHs"], rel=1e-3)
    assert sh["kernel_GHs"] > 20 and 1500 < sh["sclk_mhz"] < 2600
