import sys, time, json
sys.path.insert(0, 'bitcoin-miner_amd')
import gpuhash
with gpuhash.Engine([0]) as e:
    for name, m, lo, n in [("d11 J4 q4", b"bradfitz", 10**10, 1 << 34), ("d12 J5 q1", b"bradfitz", 10**11, 1 << 34),
                           ("d13 J5 q2", b"bradfitz", 10**12, 1 << 34), ("d10 J4 q3", b"bradfitz", 10**9, 1 << 31),
                           ("d9 J4 q2", b"bradfitz", 10**8, 1 << 29)]:
        e.min(m, lo, lo + n - 1)
        best = 1e9
        for _ in range(3):
            t = time.perf_counter(); e.min(m, lo, lo + n - 1); best = min(best, time.perf_counter() - t)
        l = max(e.launches(), key=lambda x: x["nonces"])
        print(json.dumps({"case": name, "GHs": round(n / best / 1e9, 3), "J": l["J"], "sclk": round(l["sclk_mhz"])}), flush=True)
