"""GPU: the task pipeline's transfer primitives -- CU-masked streams (taxi2_stream_create_cus) and
the text copy into pinned host memory (taxi2_copy_text_dev) -- on their own, byte for byte."""

from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_cu_stream_ranges_and_work(engine):
    import torch

    from taxi2_amd._native import NativeError

    ncu = engine.num_cus()
    assert ncu > 0
    for first, count in ((0, 0), (-1, 4), (ncu - 2, 4)):
        with pytest.raises(NativeError):
            engine.cu_stream(first, count)
    dev = torch.device("cuda", engine.device)
    hs = [engine.cu_stream(0, min(8, ncu)), engine.cu_stream(min(8, ncu - 1), ncu - min(8, ncu - 1))]
    try:
        x = torch.arange(1 << 20, dtype=torch.int64, device=dev)
        outs = []
        for h in hs:
            s = torch.cuda.ExternalStream(h, device=dev)
            s.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(s):
                outs.append((x * 3 + 1).sum())
            s.synchronize()
        want = 3 * ((1 << 20) * ((1 << 20) - 1) // 2) + (1 << 20)
        assert [int(o) for o in outs] == [want, want]
    finally:
        for h in hs:
            engine.destroy_stream(h)


@pytest.mark.parametrize("nbytes,offset", [(1, 0), (15, 0), (16, 0), (4097, 0), ((3 << 20) + 5, 0), (1000, 3)])
def test_copy_text_dev_exact(engine, nbytes, offset):
    import torch

    from taxi2_amd._native import NativeError

    dev = torch.device("cuda", engine.device)
    rng = np.random.default_rng(nbytes)
    src_h = rng.integers(0, 256, nbytes + offset, dtype=np.uint8)
    src = torch.as_tensor(src_h, device=dev)
    dst = torch.zeros(nbytes + 32, dtype=torch.uint8, pin_memory=True)
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    # offset 3: an unaligned source takes the DMA path
    engine.copy_text_dev(src.data_ptr() + offset, dst.data_ptr(), nbytes, s.cuda_stream)
    s.synchronize()
    got = dst.numpy()
    assert np.array_equal(got[:nbytes], src_h[offset:offset + nbytes])
    assert not got[nbytes:].any()  # nothing written past the end
    with pytest.raises(NativeError):  # pageable host memory is refused
        engine.copy_text_dev(src.data_ptr(), np.zeros(16, np.uint8).ctypes.data, 16, s.cuda_stream)
