"""Summary of the last A/B session's outputs under gpurun_out/ (lab tool)."""
import json
import os
import sys

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")


def objs(path):
    txt = open(path).read()
    dec, i = json.JSONDecoder(), 0
    while i < len(txt):
        while i < len(txt) and txt[i].isspace():
            i += 1
        if i >= len(txt):
            break
        o, i = dec.raw_decode(txt, i)
        yield o


def main():
    p = os.path.join(OUT, "ab_env.jsonl")
    if os.path.exists(p):
        for o in objs(p):
            pr = o.get("probe", {})
            print(o.get("set", "")[-24:].ljust(24), {k: v["us"] for k, v in pr.items() if isinstance(v, dict) and "us" in v})
    p = os.path.join(OUT, "stamp_kpart.json")
    if os.path.exists(p) and os.path.getsize(p):
        for k, v in json.load(open(p)).items():
            print(k, v.get("graph_us"), "loop", v.get("loop_start"), v.get("loop_end"), "exit", v.get("exit"))
            for r in v.get("slowest_wg_waves", []):
                print("   ", r)
    p = os.path.join(OUT, "stamp_stream.json")
    if os.path.exists(p) and os.path.getsize(p):
        for k, v in json.load(open(p)).items():
            print(k, v)


if __name__ == "__main__":
    main()
