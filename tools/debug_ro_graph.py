"""Debug: the eager part of test_reference_order_in_a_replayed_graph, printing mismatches."""
import os, random, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np, torch
import oracle_ffi as O
from e2sar_amd import sar, _capi

def main(on_cap):
    rnd = random.Random(5)
    mp = O.max_pld_len(1500)
    stride = (36 + mp + 15) // 16 * 16
    seqs = []
    for k in range(8):
        ev = np.random.default_rng(900 + k).integers(0, 256, 150_000 + 7_777 * k, dtype=np.uint8)
        pk, ln = O.segment_event(ev, 40 + k, 4321, 1, 2, 2, mp, stride)
        order = list(range(len(ln)))
        if k % 3 == 1:
            rnd.shuffle(order)
        seqs.append([(pk[i], int(ln[i])) for i in order])
    out = []
    while any(seqs):
        s = rnd.choice([s for s in seqs if s])
        out.append(s.pop(0))
    pk = np.stack([p for p, _ in out]); ln = np.array([L for _, L in out], np.uint32)
    r = O.Reassembler(True, 1 << 20); r.set_time(100); r.push_batch(pk, ln)
    ref = {}
    for b, e, d in r.pop_all():
        ref.setdefault((e, d), []).append(b)
    ctx = sar.Context(0)
    n = len(ln)
    dpk = torch.from_numpy(np.ascontiguousarray(pk).reshape(-1)).to(ctx.torch_device)
    dln = torch.from_numpy(ln.view(np.int32).copy()).to(ctx.torch_device)
    R = sar.DeviceReassembler(ctx, with_lb_header=True, table_slots=256, queue_capacity=1024, lost_capacity=1024,
                              arena_bytes=64 << 20, flags=_capi.REAS_REFERENCE_ORDER)
    st = torch.cuda.Stream() if on_cap else None
    with torch.cuda.stream(st) if st is not None else torch.cuda.stream(torch.cuda.current_stream()):
        R.recycle(force=True, stream=st)
        R.reassemble(dpk, stride, dln, n, stream=st, now_ms=100)
    torch.cuda.synchronize()
    got = {}
    for rec in R.poll():
        got.setdefault((rec.eventNum, rec.dataId), []).append(R.event_bytes(rec))
    print("on_cap", on_cap, "ref keys", sorted(ref), "got keys", sorted(got))
    for k in sorted(set(ref) | set(got)):
        a = sorted(ref.get(k, [])); b = sorted(got.get(k, []))
        if a != b:
            print(" key", k, "ref", [len(x) for x in a], "got", [len(x) for x in b])
            for x, y in zip(a, b):
                if len(x) == len(y):
                    xa = np.frombuffer(x, np.uint8); ya = np.frombuffer(y, np.uint8)
                    bad = np.nonzero(xa != ya)[0]
                    print("   first bad bytes", bad[:10], "count", len(bad))
    print("stats", {f: getattr(R.stats(), f) for f in ("eventSuccess", "totalPackets", "dataErrCnt", "badHeaderDiscards", "inProgress", "errorFlags")}, r.stats())

if __name__ == "__main__":
    main(False); main(True)
