import sys, time, json
sys.path.insert(0, 'bitcoin-miner_amd')
import gpuhash
with gpuhash.Engine([0]) as e:
    for rc in [400, 1000, 2000, 4000, 400, 1000, 2000, 4000]:
        e.min(b"bradfitz", 0, (1 << 32) - 1, rchunk=rc)
        ts = []
        for _ in range(4):
            t = time.perf_counter(); r = e.min(b"bradfitz", 0, (1 << 32) - 1, rchunk=rc); ts.append(time.perf_counter() - t)
        print(json.dumps({"gmax": rc, "GHs": round((1 << 32) / min(ts) / 1e9, 3), "res": list(r)}), flush=True)
