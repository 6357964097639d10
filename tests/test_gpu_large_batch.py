"""reassemble_batch on a batch larger than the Infinity Cache (BASELINE config 3's 64K
datagram launches: 70 x 8 MiB at MTU 9000 = 590 MB of slots) takes the split form
internally (classify + one-round scatter); every event must come back byte-exact with
every counter as for a fused launch."""
import pytest

pytestmark = pytest.mark.gpu


def test_config3_sized_launch_round_trip(hip):
    import torch
    from e2sar_amd import sar
    E, B = 70, 8 << 20
    g = torch.Generator(device=hip.torch_device)
    g.manual_seed(0xC3)
    src = torch.randint(0, 256, (E, B), dtype=torch.uint8, device=hip.torch_device, generator=g)
    seg = sar.DeviceSegmenter(hip, mtu=9000, lb_hdr_version=3)
    plan = seg.plan([(src[i].data_ptr(), B, 7000 + i, 4321, 1 + i, (1 << 48) + i) for i in range(E)])
    assert plan.total_packets == E * 939 and plan.total_packets * seg.stride > (320 << 20)
    pk, ln = seg.alloc_packets(plan.total_packets)
    seg.segment(plan, pk, ln)
    R = sar.DeviceReassembler(hip, with_lb_header=True, table_slots=1024, queue_capacity=256,
                              arena_bytes=E * B + 4096)
    for rep in range(2):
        R.reassemble(pk, seg.stride, ln, plan.total_packets)
        torch.cuda.synchronize()
        recs = R.poll()
        st = R.stats()
        assert len(recs) == E and int(st.eventSuccess) == E and int(st.inProgress) == 0
        assert int(st.totalPackets) == plan.total_packets and int(st.errorFlags) == 0
        assert int(st.badHeaderDiscards) == 0 and int(st.dataErrCnt) == 0
        arena = R.arena_tensor()
        for r in recs:
            assert r.numFragments == 939
            assert torch.equal(arena[r.arenaOffset: r.arenaOffset + B], src[r.eventNum - 7000]), (rep, r.eventNum)
        R.recycle(force=True)
        R.reset_stats()
