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


@pytest.mark.parametrize("pinned", [False, True])
def test_streamer_prefetch_at_chunk_boundaries(pinned):
    """The online job's pattern (train/online.py): feed chunk 0, consume it; feed chunk 1 and
    prefetch() (its first batches copy while the job validates); slow compute on the consumer
    stream; consume chunk 1; feed chunk 2 + prefetch; consume chunk 2. Every batch arrives
    exactly once, in its chunk, in order, with its bytes — no batch skipped, duplicated or
    overwritten at a boundary (round-4 ADVICE: only feed-after-drain was covered)."""
    from wellflow.data.stream import DeviceStreamer

    chunks = [_batches(n, B=2048, seed=10 + c, pinned=pinned) for c, n in enumerate((8, 5, 9))]
    st = DeviceStreamer(None, DEV, depth=4)
    big = torch.randn(2048, 2048, device=DEV)
    got = []
    for c, src in enumerate(chunks):
        if c == 0:
            st.feed(src)
        mine = []
        for slot in st:
            xd, yd = st.slots[slot][0], st.slots[slot][1]
            mine.append((xd.clone(), yd.clone()))  # copies queued on the consumer stream
        got.append(mine)
        if c + 1 < len(chunks):
            st.feed(chunks[c + 1])
            st.prefetch()
            for _ in range(20):  # "validation": slow work while the next chunk's copies run
                big = torch.tanh(big @ big * 1e-3)
    torch.cuda.synchronize()
    for c, (mine, src) in enumerate(zip(got, chunks)):
        assert len(mine) == len(src), (c, len(mine), len(src))
        for i, ((xd, yd), (x, y)) in enumerate(zip(mine, src)):
            assert torch.equal(xd.cpu(), x) and torch.equal(yd.cpu(), y), (c, i)
