"""Per-layer budget of the BatchNorm backward from a tools/tapeprof.py --csv file (one training
step's launches, side stream off, median per launch):

    python tools/bn_layers.py <tapeprof.csv> --es 2 [--md out.md]

For each BN layer (the program op whose BatchNorm it is): rows M, channels C, the BN-backward launch entries and their
kernels, microseconds, the bytes those kernels move (passes over [M][C] at the storage element size: seg_bn_backward
reads dA and y twice and writes dY = 5 passes; the apply after a producer-epilogue reduction 3 passes; the tile
finalize ~0) and the achieved GB/s against 5 TB/s (a streaming pass's practical rate on MI355X), then the time above
that floor summed by size bucket (<= 65k rows, larger).  A BNOUT layer's reduction runs inside the epilogue of
the data gradient that completes its dA and is not separable here.
"""
import argparse
import collections
import csv

PASSES = {"seg_bn_backward": 5, "seg_bn_bwd_apply": 3, "seg_bn_bwd_finalize_tiles": 0}
KERNELS = {"seg_bn_backward": 3, "seg_bn_bwd_apply": 1, "seg_bn_bwd_finalize_tiles": 1}
FLOOR_GBS = 5000.0


def base(entry):
    for k in PASSES:
        if entry == k or entry.startswith(k + "_"):
            return k
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--es", type=int, default=2, help="storage bytes per element (2 bf16io, 4 f32)")
    ap.add_argument("--md", default=None)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    layers = collections.OrderedDict()
    for r in rows:
        b = base(r["entry"])
        if b is None or not r["label"].endswith(":bwd"):
            continue
        k = int(r["label"].split(":")[0])
        L = layers.setdefault(k, {"M": int(r["M_out"]), "C": int(r["cout"]), "kind": r["kind"], "ks": r["ks"],
                                  "cin": r["cin"], "entries": [], "us": 0.0, "bytes": 0, "kernels": 0})
        L["entries"].append(b)
        L["us"] += float(r["us"])
        L["bytes"] += PASSES[b] * L["M"] * L["C"] * a.es
        L["kernels"] += KERNELS[b]
    out = ["# BatchNorm backward per layer (one training step, side stream off, tools/tapeprof.py medians)", "",
           f"{len(layers)} BN layers; storage {a.es} bytes/element; floor = the layer's pass bytes at "
           f"{FLOOR_GBS / 1e3:.0f} TB/s.", "",
           "| op | conv | rows | C | entries (kernels) | us | bytes | GB/s | floor us | above floor us |",
           "|---|---|---|---|---|---|---|---|---|---|"]
    buckets = collections.defaultdict(lambda: [0, 0.0, 0.0, 0])
    tot_us = tot_floor = 0.0
    for k, L in sorted(layers.items(), key=lambda kv: -kv[1]["us"]):
        floor = L["bytes"] / (FLOOR_GBS * 1e3)
        gbs = L["bytes"] / L["us"] / 1e3 if L["us"] else 0.0
        ent = " + ".join(e.replace("seg_bn_", "") for e in L["entries"])
        out.append(f"| {k} | {L['kind']} k{L['ks']} {L['cin']}->{L['C']} | {L['M']} | {L['C']} | {ent} ({L['kernels']}) "
                   f"| {L['us']:.1f} | {L['bytes'] / 1e6:.1f} MB | {gbs:.0f} | {floor:.1f} | {L['us'] - floor:.1f} |")
        bk = "<= 65k rows" if L["M"] <= 65536 else "> 65k rows"
        bb = buckets[bk]
        bb[0] += 1
        bb[1] += L["us"]
        bb[2] += floor
        bb[3] += L["kernels"]
        tot_us += L["us"]
        tot_floor += floor
    out += ["", "| bucket | layers | kernels | us | floor us | above floor us |", "|---|---|---|---|---|---|"]
    for bk, (n, us, fl, nk) in sorted(buckets.items()):
        out.append(f"| {bk} | {n} | {nk} | {us:.0f} | {fl:.0f} | {us - fl:.0f} |")
    out.append(f"| all | {len(layers)} | {sum(b[3] for b in buckets.values())} | {tot_us:.0f} | {tot_floor:.0f} | "
               f"{tot_us - tot_floor:.0f} |")
    text = "\n".join(out) + "\n"
    if a.md:
        with open(a.md, "w") as fh:
            fh.write(text)
    print(text)


if __name__ == "__main__":
    main()
