"""Generate tests/golden/sar_golden.json from the CPU oracle.

Run:  python tests/golden/make_golden.py

The vectors are oracle outputs.  The oracle itself is pinned by the reference's own
known answers (see tests/test_oracle_golden.py, which checks these fixtures AND those
known answers); the large cases are stored as header hexes + SHA-256 digests so the
fixture stays small.  The reference engines cannot be built in this image (Boost/gRPC
absent), so no vector here was produced by running reference code.
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import oracle_ffi as O  # noqa: E402
import sar_inputs as S  # noqa: E402

SEND_STR = b"THIS IS A VERY LONG EVENT MESSAGE WE WANT TO SEND EVERY 1 SECONDS."


def datagram_stream_digest(pk, ln):
    h = hashlib.sha256()
    for k in range(len(ln)):
        h.update(pk[k, : int(ln[k])].tobytes())
    return h.hexdigest()


def seg_case(name, nbytes, mtu, ver, n_events=1):
    mp = O.max_pld_len(mtu)
    out = {"name": name, "bytes": nbytes, "mtu": mtu, "lbHdrVersion": ver, "maxPldLen": mp,
           "events": []}
    for i in range(n_events):
        ev = S.event_bytes(i, nbytes)
        pk, ln = O.segment_event(ev, i, S.DATA_ID, S.entropy(i), S.lb_tick(i), ver, mp)
        out["events"].append({
            "eventNum": i, "dataId": S.DATA_ID, "entropy": S.entropy(i), "lbTick": S.lb_tick(i),
            "event_sha256": hashlib.sha256(ev.tobytes()).hexdigest(),
            "numPackets": int(len(ln)),
            "first_hdr": pk[0, :36].tobytes().hex(),
            "second_hdr": pk[1, :36].tobytes().hex() if len(ln) > 1 else None,
            "last_hdr": pk[-1, :36].tobytes().hex(),
            "last_len": int(ln[-1]),
            "datagrams_sha256": datagram_stream_digest(pk, ln),
        })
    return out


def full_case(name, payload, mtu, ver, event_num, data_id, entropy, tick):
    mp = O.max_pld_len(mtu)
    pk, ln = O.segment_event(np.frombuffer(payload, np.uint8), event_num, data_id, entropy, tick, ver, mp)
    return {"name": name, "mtu": mtu, "lbHdrVersion": ver, "eventNum": event_num, "dataId": data_id,
            "entropy": entropy, "lbTick": tick, "payload_hex": payload.hex(),
            "datagrams_hex": [pk[k, : int(ln[k])].tobytes().hex() for k in range(len(ln))]}


def reas_case(name, dgrams, with_lb, ring=0):
    """ring 0: the reference's unbounded eventQueue (hpp:126-127); ring > 0: the device's
    completed-record ring of that capacity (e2sar_hip_reas_config.queueCapacity), a
    parameter of this build -- not reference behaviour"""
    r = O.Reassembler(with_lb, ring)
    for d in dgrams:
        r.push(d)
    evs = r.pop_all()
    c = {"name": name, "withLBHeader": with_lb,
            "datagrams_hex": [d.hex() for d in dgrams],
            "events": [{"eventNum": e, "dataId": d, "hex": b.hex()} for b, e, d in evs],
            "stats": r.stats()}
    if ring:
        c["deviceRingCapacity"] = ring
    return c


def main():
    g = {"generator": "tests/golden/make_golden.py (oracle/e2sar_oracle.c)", "segment": [], "segment_full": [],
         "reassemble": []}
    # (i) the reference test string at the MTUs its tests use
    for mtu in (80, 104, 1500):
        for ver in (2, 3):
            g["segment_full"].append(full_case(f"send_str_mtu{mtu}_v{ver}", SEND_STR, mtu, ver, 0, 4321, 0xBEEF,
                                               0x0123456789ABCDEF))
    # (ii)/(iii) large seeded events: headers + digests
    g["segment"].append(seg_case("A_1MiB_mtu1500_v2", 1 << 20, 1500, 2, 2))
    g["segment"].append(seg_case("A_1MiB_mtu1500_v3", 1 << 20, 1500, 3, 1))
    g["segment"].append(seg_case("B_1MiB_mtu9000_v2", 1 << 20, 9000, 2, 1))
    g["segment"].append(seg_case("B_1MiB_mtu9000_v3", 1 << 20, 9000, 3, 1))
    g["segment"].append(seg_case("C_8MiB_mtu9000_v3", 8 << 20, 9000, 3, 1))
    g["segment"].append(seg_case("frames_100000B_mtu1500_v2", 100000, 1500, 2, 1))

    # (iv) reassembly vectors
    mp = O.max_pld_len(80)
    evs = [S.event_bytes(100 + i, 67) for i in range(3)]
    dg = []
    for i, ev in enumerate(evs):
        pk, ln = O.segment_event(ev, i, 4321, 7, 99, 2, mp)
        dg.append([pk[k, : int(ln[k])].tobytes() for k in range(len(ln))])
    in_order = [d for e in dg for d in e]
    g["reassemble"].append(reas_case("mtu80_in_order_lb", in_order, True))
    shuffled = [dg[0][0], dg[1][0], dg[2][0], dg[2][3], dg[0][4], dg[1][2], dg[0][1], dg[2][1], dg[1][4],
                dg[0][3], dg[2][4], dg[1][1], dg[0][2], dg[2][2], dg[1][3]]
    g["reassemble"].append(reas_case("mtu80_interleaved_offset0_first_lb", shuffled, True))
    late0 = [dg[0][1], dg[0][0], dg[0][2], dg[0][3], dg[0][4]]
    g["reassemble"].append(reas_case("mtu80_late_offset0_quirk_lb", late0, True))
    dup = [dg[1][0], dg[1][1], dg[1][1], dg[1][2], dg[1][3], dg[1][4]]
    g["reassemble"].append(reas_case("mtu80_duplicate_fragment_lb", dup, True))
    badv = list(dg[2])
    b = bytearray(badv[2]); b[16] = 0x20; badv[2] = bytes(b)
    g["reassemble"].append(reas_case("mtu80_bad_version_lb", badv, True))
    nolb = [d[16:] for d in dg[0]]
    g["reassemble"].append(reas_case("mtu80_no_lb_header", nolb, False))
    g["reassemble"].append(reas_case("mtu80_device_ring_cap2_lb", in_order, True, ring=2))

    path = os.path.join(HERE, "sar_golden.json")
    with open(path, "w") as f:
        json.dump(g, f, indent=1, sort_keys=True)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
