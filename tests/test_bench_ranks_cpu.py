"""CPU: bench.py's torchrun path (main_ranks) end to end over world-size-2 gloo, with the
HIP engine replaced by an oracle-backed stand-in and torch.cuda by a two-GPU fake -- the
code the driver's N > 1 scaling run executes (timed steps, the ranks' search leg with
its gloo merge, rank 0's in-process repeat over all GPUs, the device/PCI checks, the one
JSON line) with no GPU.  The stand-in is test infrastructure: it hashes with the C
oracle on the search range (config 1's [0, 9999], whose golden is committed) and answers
the 2^32 step windows, which the oracle could not scan here, from the committed CPU
goldens that cover them."""
import io
import json
import os
import socket
import sys
import types

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, ndev, share, q, pinned=False):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "bitcoin-miner_amd"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    if share:
        os.environ["GPUHASH_SHARE_GPU"] = "1"
    if pinned:  # the launcher gave each rank one visible GPU: every rank sees ordinal 0
        os.environ["HIP_VISIBLE_DEVICES"] = str(rank)
    import torch
    import gpuhash
    import hash_oracle
    import bench
    oracle = hash_oracle.load_c_oracle()
    import json
    with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as f:
        goldens = json.load(f)["ranges"]

    class FakeEngine:
        """gpuhash.Engine's surface, oracle-backed on small ranges."""

        def __init__(self, devices=None, lib_path=None):
            self.devs = list(devices)
            self.recs = []

        def min(self, msg, lo, hi):
            cuts = gpuhash.shard_range(len(msg), lo, hi, len(self.devs))  # the real planner
            self.recs = [{"device": self.devs[i], "J": 4, "C2": 0, "EX": 0, "digits": 10, "c": 1,
                          "shard": i, "stream_device": self.devs[i], "lo": c[0], "hi": c[1],
                          "nonces": c[1] - c[0] + 1, "ms": 1e-6 * (c[1] - c[0] + 1), "sclk_mhz": 2400.0}
                         for i, c in enumerate(cuts) if c is not None]
            if hi - lo < 1_000_000:
                return oracle.min(msg, lo, hi)
            # a 2^32 step window: the committed CPU golden of a range that contains it and
            # whose winner lies inside it is this window's answer too (its min over the
            # superset is attained here)
            for g in goldens:
                if g["msg_hex"] == msg.hex() and g["lower"] <= lo and hi <= g["upper"] and lo <= g["nonce"] <= hi:
                    return (g["hash"], g["nonce"])
            raise AssertionError(f"no golden covers [{lo}, {hi}]")

        def launches(self):
            return list(self.recs)

        @property
        def ndevices(self):
            return len(self.devs)

        def close(self):
            pass

        def __enter__(self):
            return self

        def __exit__(self, *exc):
            pass

    gpuhash.Engine = FakeEngine
    # a physical GPU's PCI id: by ordinal, or by rank when each rank sees only its own GPU
    props = lambda d: types.SimpleNamespace(pci_domain_id=0, pci_bus_id=0x10 + 0x10 * (rank if pinned else d),
                                            pci_device_id=0)
    torch.cuda.device_count = lambda: ndev
    torch.cuda.set_device = lambda d: None
    torch.cuda.synchronize = lambda d=None: None
    torch.cuda.get_device_properties = props
    args = types.SimpleNamespace(gpus=world, steps=2, warmup=1, no_cpu_baseline=True, cpu_seconds=1.0,
                                 config="2", inproc=None, search=(0, 9999), no_search=False)
    out, err = io.StringIO(), io.StringIO()
    sys.stdout, sys.stderr = out, err
    code = 0
    try:
        bench.main_ranks(args, world, rank, rank)
    except SystemExit as e:
        code = e.code
    sys.stdout, sys.stderr = sys.__stdout__, sys.__stderr__
    q.put((rank, code, out.getvalue(), err.getvalue()))


def _run(ndev, share, pinned=False):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, ndev, share, q, pinned)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, (c, o, e)) for r, c, o, e in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(timeout=30)
    code, text, err = res[0]
    line = json.loads([x for x in text.splitlines() if x.startswith("{")][-1])
    _run.stderr = err
    return code, line


def test_two_ranks_on_two_gpus_search_leg_and_inproc_repeat():
    code, line = _run(ndev=2, share=False)
    assert code in (0, None), line.get("device_check")
    assert line["n_gpus"] == 2 and line["config"]["parallelism"] == "dp2"
    s = line["search_2p40"]
    # each rank searched its cost-balanced window of [0, 9999]; gloo merge = config 1's golden
    assert s["golden_name"] == "cfg1_bradfitz_9999" and s["matches_golden"] is True
    assert tuple(s["result"]) == (1419516646206828, 9898)
    assert [x["shard"] for x in s["shards"]] == [0, 1] and [x["device"] for x in s["shards"]] == [0, 1]
    assert s["shards"][0]["pci"] != s["shards"][1]["pci"]
    # rank 0's in-process repeat over devices [0, 1], same golden
    si = line["search_2p40_inproc"]
    assert si["matches_golden"] is True and si["devices"] == [0, 1]
    assert [x["device"] for x in si["shards"]] == [0, 1]
    assert [(d["rank"], d["device"], d["pci"]) for d in line["rank_devices"]] == \
        [(0, 0, "0000:10:00"), (1, 1, "0000:20:00")]
    assert "device_check" not in line
    # same-run scaling evidence: rank 0's search window again, alone
    sc = s["scaling"]
    assert sc["shard"] == 0 and sc["windows"] == s["shards"][0]["windows"]
    assert sc["t_all_s"] == s["seconds"] and sc["scaling_efficiency"] > 0
    # the timed step spans [0, 2^33): checked against config 2's N = 2 golden
    assert line["matches_golden"] is True and line["result_check"]["golden_names"] == ["cfg2_bradfitz_2gpu"]
    # a run over distinct GPUs says so in one stderr line
    summ = [x for x in _run.stderr.splitlines() if "distinct GPUs" in x]
    assert len(summ) == 1, _run.stderr
    assert "2 distinct GPUs (search_2p40)" in summ[0] and "0000:10:00" in summ[0] and "0000:20:00" in summ[0]
    assert f"scaling_efficiency {sc['scaling_efficiency']}" in summ[0] and "MHz" in summ[0]


def test_ranks_pinned_to_one_visible_gpu_each():
    """ranks launched with one visible GPU each all report ordinal 0; distinct
    GPUs are judged by (host, PCI id), so a correct pinned run has no device_check."""
    code, line = _run(ndev=1, share=False, pinned=True)
    assert code in (0, None), line.get("device_check")
    assert [d["device"] for d in line["rank_devices"]] == [0, 0]
    assert len({d["pci"] for d in line["rank_devices"]}) == 2
    assert "device_check" not in line
    assert line["search_2p40"]["matches_golden"] is True
    assert "search_2p40_inproc" not in line  # no rank can see every GPU


def test_shared_gpu_rehearsal_repeats_ordinal_zero():
    code, line = _run(ndev=1, share=True)
    assert code in (0, None)
    assert line["search_2p40"]["matches_golden"] is True
    assert line["search_2p40_inproc"]["devices"] == [0, 0]
    assert "device_check" not in line
    assert "distinct GPUs" not in _run.stderr  # one physical GPU: no summary
