"""Generate tests/golden/combined_dataset_routing.json from the REFERENCE's own
src/CombinedDataset.py (run in the build container only; never on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_data_golden.py

cv2 / albumentations are not installed, so empty stand-in modules are
registered for the per-source readers' imports, and the three reader classes
the reference constructs are replaced (inside the loaded module) by fixed-size
stand-ins that return their index.  Everything else -- random.seed, the
shuffles, the validation split and __getitem__'s routing -- is the reference's
own code (src/CombinedDataset.py:8-205).
"""
from __future__ import annotations

import importlib.util
import json
import os
import sys
import types

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("SEG_REFERENCE", "/root/reference")

CASES = [  # (bdd100k, sea, carla, val_split, seed)
    (7, 5, 3, 0.0, 42), (7, 5, 3, 0.3, 42), (20, 0, 6, 0.25, 42), (0, 9, 4, 0.5, 7), (11, 13, 0, 0.2, 42),
    (40, 25, 15, 0.2, 123),
]


def _stub(name):
    m = types.ModuleType(name)
    def attr(name):
        if name.startswith("__"):
            raise AttributeError(name)
        return lambda *a, **k: None
    m.__getattr__ = attr
    return m


def load_reference_combined():
    for name in ("cv2", "albumentations", "albumentations.pytorch"):
        sys.modules.setdefault(name, _stub(name))
    sys.modules["albumentations"].pytorch = sys.modules["albumentations.pytorch"]
    src = types.ModuleType("src")
    src.__path__ = [os.path.join(REF, "src")]
    sys.modules.setdefault("src", src)
    spec = importlib.util.spec_from_file_location("src.CombinedDataset", os.path.join(REF, "src", "CombinedDataset.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


class _Source:
    def __init__(self, tag, n):
        self.tag, self.n, self.is_train = tag, n, True

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        return (self.tag, i)


def main():
    mod = load_reference_combined()
    out = []
    for nb, ns, nc, vs, seed in CASES:
        mod.BDD100KDataset = lambda **k: _Source("bdd100k", nb)
        mod.SEAMEDataset = lambda **k: _Source("sea", ns)
        mod.CarlaDataset = lambda **k: _Source("carla", nc)
        cfg = {"img_dir": "-", "mask_dir": "-", "annotation_file": "-"}  # contents unused by the stand-ins
        ds = mod.CombinedLaneDataset(bdd100k_config=cfg if nb else None, sea_config=cfg if ns else None,
                                     carla_config=cfg if nc else None, val_split=vs, seed=seed)
        tr = ds.get_train_dataset()
        train = [list(tr[i]) for i in range(len(tr))]
        va = ds.get_val_dataset()
        val = [list(va[i]) for i in range(len(va))]
        out.append({"bdd100k": nb, "sea": ns, "carla": nc, "val_split": vs, "seed": seed,
                    "train_size": ds.train_size, "val_size": ds.val_size, "train": train, "val": val})
    with open(os.path.join(HERE, "combined_dataset_routing.json"), "w") as f:
        json.dump(out, f)
    print(f"wrote {len(out)} cases")


if __name__ == "__main__":
    main()
