"""DeviceStreamer (data/stream.py): the producer thread's ring delivers every batch of a
source exactly once, in order, with the right bytes, while the consumer keeps overwriting
nothing it has not finished with — for pinned and pageable sources and across feed()."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _batches(n, B=4096, F=16, seed=0, pinned=False):
    g = torch.Generator().manual_seed(seed)
    out = []
    for _ in range(n):
        x = torch.randn(B, F, generator=g)
        y = torch.randn(B, generator=g)
        if pinned:
            x, y = x.pin_memory(), y.pin_memory()
        out.append((x, y))
    return out


@pytest.mark.parametrize("pinned", [False, True])
@pytest.mark.parametrize("depth", [3, 4])
def test_streamer_delivers_every_batch_in_order(pinned, depth):
    from wellflow.data.stream import DeviceStreamer

    src = _batches(11, pinned=pinned)
    st = DeviceStreamer(src, DEV, depth=depth)
    acc = torch.zeros(1, device=DEV)
    got = []
    for slot in st:
        xd, yd = st.slots[slot][0], st.slots[slot][1]
        # consumer work on the stream the ring orders against (a slow-ish kernel sequence)
        for _ in range(3):
            acc += xd.float().sum() * 1e-9
        got.append((xd.clone(), yd.clone()))
    torch.cuda.synchronize()
    assert len(got) == len(src)
    for (xd, yd), (x, y) in zip(got, src):
        assert torch.equal(xd.cpu(), x) and torch.equal(yd.cpu(), y)


def test_streamer_feed_second_source_and_bf16_cast():
    from wellflow.data.stream import DeviceStreamer

    st = DeviceStreamer(None, DEV, depth=3, x_dtype=torch.bfloat16)
    for seed, n in ((1, 5), (2, 7)):
        src = _batches(n, seed=seed)
        st.feed(src)
        seen = 0
        for i, slot in enumerate(st):
            xd = st.slots[slot][0]
            assert xd.dtype == torch.bfloat16
            assert torch.equal(xd.cpu(), src[i][0].to(torch.bfloat16))
            seen += 1
        assert seen == n
    st.close()
