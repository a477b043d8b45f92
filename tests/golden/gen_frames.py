"""Generate tests/golden/golden_frames.json: Frame specs with their
Frame.Marshal bytes and Frame.Hash under the oracle's ugorji restatement
(oracle/gosemantics.py).  Data only; regenerate with
    python tests/golden/gen_frames.py
PARITY UNPINNED (no Go / ugorji here): the fixture freezes the restatement so
any change to either encoder is caught."""
import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import gosemantics as gs  # noqa: E402
from tests.frame_spec import frame_spec, to_types  # noqa: E402


def main():
    rng = random.Random(20260)
    out = []
    for i in range(24):
        spec = frame_spec(rng)
        if i == 0:  # the empty frame
            spec = {"Round": 0, "Peers": None, "Roots": None, "Events": None, "PeerSets": None, "Timestamp": 0}
        if i == 1:  # empty (non-nil) collections and int-key ordering 9 < 10 < 100
            spec.update(Peers=[], Roots={}, Events=[], PeerSets={10: [], 9: None, 100: [], -1: []})
        f = to_types(spec, gs)
        raw = gs.frame_marshal(f)
        spec_json = dict(spec)
        if spec_json["PeerSets"] is not None:
            spec_json["PeerSets"] = {str(k): v for k, v in spec_json["PeerSets"].items()}
        out.append({"spec": spec_json, "marshal": raw.hex(), "hash": gs.SHA256(raw).hex()})
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden_frames.json")
    with open(path, "w") as fh:
        json.dump(out, fh, indent=0)
    print(f"wrote {len(out)} frames to {path}")


if __name__ == "__main__":
    main()
