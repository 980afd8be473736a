"""Graph build timing on a full-size config (diagnostic): generate the config's
stand-in on the device as bench.py does, hand torch's cached blocks back, build
the graph handle, print the create wall time and nlp_graph_build_phases.
NLP_BUILD_TRACE=1 adds every build allocation on stderr.

    python tools/create_probe.py [--config C4-sk-2005] [--repeat 2]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import nlp_loader  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C4-sk-2005")
    ap.add_argument("--repeat", type=int, default=2)
    ap.add_argument("--envs", default="", help="';'-separated NAME=VALUE[,NAME=VALUE] sets, one create each (A/B runs)")
    args = ap.parse_args()
    import torch
    nlp = nlp_loader.load()
    gg = nlp_loader.load_sub("graphgen")
    t0 = time.time()
    off, keys, du, dw, info = gg.make_workload(args.config, "cuda")
    from bench import release_cached, HBM_CLEAR_GBS
    release_cached("graph generation")
    print(json.dumps({"config": args.config, "gen_s": time.time() - t0, "M": int(keys.numel())}), flush=True)
    sets = [x for x in args.envs.split(";") if x] or [""] * args.repeat
    for es in sets:
        for kv in (x for x in es.split(",") if x):
            k, v = kv.split("=", 1)
            os.environ[k] = v
        t0 = time.time()
        G = nlp.Graph.from_device(off, keys)
        torch.cuda.synchronize()
        dt = time.time() - t0
        print(json.dumps({"env": es, "create_s": dt, "phases_ms": G.build_phases()}), flush=True)
        free0 = torch.cuda.mem_get_info()[0]
        G.close()
        time.sleep(max(0, torch.cuda.mem_get_info()[0] - free0) / 1e9 / HBM_CLEAR_GBS)  # the driver's clear


if __name__ == "__main__":
    main()
