"""Numerics of the projection GEMM kernels (rc_gemm_bf16) against a plain PyTorch fp32 reference.

Same bf16 inputs on both sides, f32 accumulation on both sides, so f32 outputs
agree to summation-order rounding (atol/rtol 1e-4 here) and bf16 outputs to one
bf16 rounding (rtol 1e-2).  Every tile variant and every fused epilogue.
"""
import pytest

from conftest import import_pkg

pytestmark = pytest.mark.gpu

EPI_BF16, EPI_GELU, EPI_RESID, EPI_PATCH = 0, 1, 2, 3


def run(epi, variant, A, W, bias, M, out, pos=None, tokens=0):
    L = import_pkg("_lib")
    lib = L.load()
    import torch

    N, K = W.shape
    L.check(lib.rc_gemm_bf16(epi, variant, A.data_ptr(), W.data_ptr(), bias.data_ptr(), M, N, K, out.data_ptr(),
                             None if pos is None else pos.data_ptr(), tokens, torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()


@pytest.mark.parametrize("variant", [4, 8])
@pytest.mark.parametrize("M,N,K", [(300, 768, 768), (1000, 2304, 768), (513, 3072, 768), (257, 768, 3072), (64, 256, 64)])
@pytest.mark.parametrize("epi", [EPI_BF16, EPI_GELU, EPI_RESID])
def test_gemm_matches_torch_fp32(cuda, variant, M, N, K, epi):
    import torch

    g = torch.Generator(device=cuda).manual_seed(M + N + K)
    Mp = (M + 255) // 256 * 256
    A = (torch.randn(Mp, K, device=cuda, generator=g) * 0.5).to(torch.bfloat16)
    A[M:] = 0
    W = (torch.randn(N, K, device=cuda, generator=g) * 0.05).to(torch.bfloat16)
    bias = torch.randn(N, device=cuda, generator=g) * 0.1
    ref = A[:M].float() @ W.float().T + bias
    if epi == EPI_RESID:
        resid = torch.randn(Mp, N, device=cuda, generator=g)
        out = resid.clone()
        run(epi, variant, A, W, bias, M, out)
        assert torch.allclose(out[:M], resid[:M] + ref, atol=1e-4, rtol=1e-4)
        assert torch.equal(out[M:], resid[M:])  # rows >= M untouched
    else:
        out = torch.full((Mp, N), 7.0, device=cuda).to(torch.bfloat16)
        run(epi, variant, A, W, bias, M, out)
        if epi == EPI_GELU:
            ref = torch.nn.functional.gelu(ref)
        assert torch.allclose(out[:M].float(), ref, atol=2e-3, rtol=1e-2)
        assert bool((out[M:].float() == 7.0).all())


@pytest.mark.parametrize("variant", [0, 9])
@pytest.mark.parametrize("M,N,K", [(1, 768, 768), (85, 3072, 768), (86, 768, 3072), (256, 2304, 768), (17, 32, 64),
                                   (200, 3072, 768), (230, 2304, 3072)])
@pytest.mark.parametrize("epi", [EPI_BF16, EPI_GELU, EPI_RESID])
def test_skinny_gemm_matches_torch_fp32(cuda, variant, M, N, K, epi):
    """M <= 256 (the CLS rows of the last layer): auto picks the skinny kernel (variant 9).  More than
    1024 16x32 tiles take the shared-weight form (four row tiles per block): (256, 2304, 768) with full
    row groups, (200, 3072, 768) and (230, 2304, 3072) with a partial last group (1 and 3 of 4 row
    tiles below M)."""
    test_gemm_matches_torch_fp32(cuda, variant, M, N, K, epi)


@pytest.mark.parametrize("variant", [4, 8])
def test_patch_epilogue_scatter(cuda, variant):
    import torch

    n_img, npatch, H, K = 3, 196, 768, 768
    T = npatch + 1
    M = n_img * npatch
    g = torch.Generator(device=cuda).manual_seed(0)
    A = torch.zeros((M + 255) // 256 * 256, K, device=cuda).to(torch.bfloat16)
    A[:M] = (torch.randn(M, K, device=cuda, generator=g)).to(torch.bfloat16)
    W = (torch.randn(H, K, device=cuda, generator=g) * 0.05).to(torch.bfloat16)
    bias = torch.randn(H, device=cuda, generator=g)
    pos = torch.randn(T, H, device=cuda, generator=g)
    hidden = torch.full((n_img * T, H), -3.0, device=cuda)
    run(EPI_PATCH, variant, A, W, bias, M, hidden, pos, T)
    ref = (A[:M].float() @ W.float().T + bias).reshape(n_img, npatch, H) + pos[1:]
    got = hidden.reshape(n_img, T, H)
    assert torch.allclose(got[:, 1:], ref, atol=1e-4, rtol=1e-4)
    assert bool((got[:, 0] == -3.0).all())  # CLS rows are not the GEMM's



@pytest.mark.parametrize("M,K", [(5 * 197, 768), (5 * 197 + 50, 3072), (2 * 197, 768), (197 + 1, 3072)])
def test_image_aligned_tiles_match_torch_fp32(cuda, M, K):
    """Variant 10 (diagnostic builds; it lost the in-model A/B at parts = 2): 224-row tiles, tile t =
    rows [197 t, 197 t + 197), f32 residual epilogue; a ragged last image (M not a multiple of 197)
    and rows >= M untouched.  The A buffer holds 224 - 197 rows past the last tile's start (the
    model pads 256).  The product library refuses the variant."""
    import torch

    L = import_pkg("_lib")
    lib = L.load()
    if getattr(lib, "rc_diag_set_gemm_variant", None) is None:  # the product build
        dummy = torch.zeros(256, 768, dtype=torch.bfloat16, device=cuda)
        rc = lib.rc_gemm_bf16(EPI_RESID, 10, dummy.data_ptr(), dummy.data_ptr(), dummy.data_ptr(), 197, 768, 768,
                              dummy.data_ptr(), None, 197, torch.cuda.current_stream().cuda_stream)
        assert rc != 0 and b"diagnostic" in lib.rc_last_error()
        return

    N, T = 768, 197
    g = torch.Generator(device=cuda).manual_seed(M + K)
    Mp = (M + 255) // 256 * 256 + 256
    A = (torch.randn(Mp, K, device=cuda, generator=g) * 0.5).to(torch.bfloat16)
    A[M:] = 0
    W = (torch.randn(N, K, device=cuda, generator=g) * 0.05).to(torch.bfloat16)
    bias = torch.randn(N, device=cuda, generator=g) * 0.1
    ref = A[:M].float() @ W.float().T + bias
    resid = torch.randn(Mp, N, device=cuda, generator=g)
    out = resid.clone()
    L.check(lib.rc_gemm_bf16(EPI_RESID, 10, A.data_ptr(), W.data_ptr(), bias.data_ptr(), M, N, K, out.data_ptr(),
                                  None, T, torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    assert torch.allclose(out[:M], resid[:M] + ref, atol=1e-4, rtol=1e-4)
    assert torch.equal(out[M:], resid[M:])
    # the same bits as the 256-row ping-pong tile (one K order for every kernel)
    out4 = resid.clone()
    run(EPI_RESID, 4, A, W, bias, M, out4)
    assert torch.equal(out[:M], out4[:M])


def test_two_workgroup_160_row_tiles_match_pingpong(cuda):
    """M = 25 216 (a 128-image slice of a batch): the two-workgroup kernel (variant 8) takes
    160-row tiles when they need fewer row-rounds of the chip's workgroup slots (on 256 CUs one
    round of 474 tiles, against two of 591 128-row tiles).  The residual epilogue's values equal
    the ping-pong kernel's bit for bit (both accumulate K in the same 16x16x32 MFMA order) and
    fp32 to summation rounding; rows >= M stay untouched."""
    import torch

    M, N, K = 25216, 768, 768
    g = torch.Generator(device=cuda).manual_seed(160)
    Mp = (M + 255) // 256 * 256
    A = (torch.randn(Mp, K, device=cuda, generator=g) * 0.5).to(torch.bfloat16)
    A[M:] = 0
    W = (torch.randn(N, K, device=cuda, generator=g) * 0.05).to(torch.bfloat16)
    bias = torch.randn(N, device=cuda, generator=g) * 0.1
    resid = torch.randn(Mp, N, device=cuda, generator=g)
    out_w2, out_pp = resid.clone(), resid.clone()
    run(EPI_RESID, 8, A, W, bias, M, out_w2)
    run(EPI_RESID, 4, A, W, bias, M, out_pp)
    assert torch.equal(out_w2, out_pp)
    ref = A[:M].float() @ W.float().T + bias
    assert torch.allclose(out_w2[:M], resid[:M] + ref, atol=1e-4, rtol=1e-4)
    assert torch.equal(out_w2[M:], resid[M:])


def test_two_workgroup_160_row_tiles_clamp_rows_past_m(cuda):
    """M = 25 344 = 99 * 256: the 160-row tiles (159 row tiles) reach 96 rows past M, beyond the
    round_up(M, 256) = M rows the ABI asks the caller for.  The kernel clamps those A rows to row
    M - 1 (results never stored), so an A buffer of exactly M rows is enough; the outputs equal
    the ping-pong kernel's bit for bit."""
    import torch

    M, N, K = 25344, 768, 768
    g = torch.Generator(device=cuda).manual_seed(161)
    A = (torch.randn(M, K, device=cuda, generator=g) * 0.5).to(torch.bfloat16)
    W = (torch.randn(N, K, device=cuda, generator=g) * 0.05).to(torch.bfloat16)
    bias = torch.randn(N, device=cuda, generator=g) * 0.1
    resid = torch.randn(M, N, device=cuda, generator=g)
    out_w2, out_pp = resid.clone(), resid.clone()
    run(EPI_RESID, 8, A, W, bias, M, out_w2)
    run(EPI_RESID, 4, A, W, bias, M, out_pp)
    assert torch.equal(out_w2, out_pp)
    ref = A.float() @ W.float().T + bias
    assert torch.allclose(out_w2, resid + ref, atol=1e-4, rtol=1e-4)
