"""ncclBroadcast (zero-copy pull from the root, kernels/allreduce_bulk.hip broadcastKernel): every
rank's receive buffer must equal the root's send buffer byte for byte, for any root, odd sizes,
in place on the root (ncclBcast) and out of place.  In-process ranks (one launch, blockIdx.y =
rank) as the other parity tests."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [2, 3, 8])
@pytest.mark.parametrize("nbytes", [1, 15, 16, 4097, (1 << 20) + 3, 48 << 20])
def test_broadcast_bytes_exact(built, n, nbytes):
    import mscclpp_amd as m

    if nbytes == 48 << 20 and n != 8:
        pytest.skip("full size once")
    ranks = m.InProcessRanks(n, 1 << 16)
    g = torch.Generator(device="cuda").manual_seed(nbytes + n)
    for call, root in enumerate((0, n - 1, n // 2)):
        sends = [torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device="cuda", generator=g) for _ in range(n)]
        inplace = call == 2
        recvs = [s if (inplace and r == root) else torch.full_like(s, 0xA5) for r, s in enumerate(sends)]
        ref = sends[root].clone()
        ranks.broadcast(sends, recvs, root, nblocks=0 if nbytes > 4096 else 3)
        torch.cuda.synchronize()
        assert ranks.errors() == [0] * n
        for r in range(n):
            assert torch.equal(recvs[r], ref), (r, root, call)
        for r in range(n):  # the send buffers of non-roots are untouched
            if r != root and not inplace:
                assert not torch.equal(sends[r], ref) or nbytes < 4
