"""Device-resident entry points (torch tensors as HBM buffers; torch is plumbing only).

Thin wrappers over the xs_*_dev C ABI: the compute runs in the HIP kernels of
librclone_crypt.so on the tensors' device and on torch's current stream of that device.
"""
import torch

from . import _lib

BLOCK_DATA = 65536
BLOCK_HDR = 16
BLOCK_SIZE = 65552
FILE_HDR = 32


def _stream(t):
    return ctypes_void(torch.cuda.current_stream(t.device).cuda_stream)


def ctypes_void(x):
    import ctypes
    return ctypes.c_void_p(x)


def _require_gpu(*ts):
    for t in ts:
        if not t.is_cuda:
            raise ValueError("rclone_amd.device needs HIP device tensors (no CPU fallback)")
        if not t.is_contiguous():
            raise ValueError("tensors must be contiguous")


def body_size(plain_len: int) -> int:
    """Bytes of wire blocks (EncryptedSize minus the 32-byte file header)."""
    full, rem = divmod(plain_len, BLOCK_DATA)
    return full * BLOCK_SIZE + (rem + BLOCK_HDR if rem else 0)


def plain_size(body_len: int) -> int:
    full, rem = divmod(body_len, BLOCK_SIZE)
    if rem and rem <= BLOCK_HDR:
        raise ValueError("truncated block header")
    return full * BLOCK_DATA + (rem - BLOCK_HDR if rem else 0)


def nblocks_plain(plain_len: int) -> int:
    return (plain_len + BLOCK_DATA - 1) // BLOCK_DATA


def workspace(nblocks: int, device) -> torch.Tensor:
    nbytes = _lib.lib().xs_workspace_bytes(nblocks)
    return torch.empty(max(nbytes, 16), dtype=torch.uint8, device=device)


def seal_object(key: bytes, nonce0: bytes, plain: torch.Tensor, body: torch.Tensor = None,
                first_block: int = 0, ws: torch.Tensor = None) -> torch.Tensor:
    """Seal a plaintext object (uint8 tensor in HBM) into wire blocks (no 32-byte header)."""
    _require_gpu(plain)
    n = plain.numel()
    if body is None:
        body = torch.empty(body_size(n), dtype=torch.uint8, device=plain.device)
    if ws is None:
        ws = workspace(nblocks_plain(n), plain.device)
    _require_gpu(body, ws)
    assert body.numel() >= body_size(n) and ws.numel() >= _lib.lib().xs_workspace_bytes(nblocks_plain(n))
    rc = _lib.lib().xs_seal_object_dev(bytes(key), bytes(nonce0), first_block, plain.data_ptr(), n,
                                       body.data_ptr(), ws.data_ptr(), _stream(plain))
    _lib.check(rc, "xs_seal_object_dev")
    return body


def open_object(key: bytes, nonce0: bytes, body: torch.Tensor, plain: torch.Tensor = None,
                ok: torch.Tensor = None, first_block: int = 0, ws: torch.Tensor = None):
    """Open wire blocks; returns (plaintext tensor, ok uint8 tensor per block)."""
    _require_gpu(body)
    m = body.numel()
    n = plain_size(m)
    nb = (m + BLOCK_SIZE - 1) // BLOCK_SIZE
    if plain is None:
        plain = torch.empty(max(n, 16), dtype=torch.uint8, device=body.device)
    if ok is None:
        ok = torch.empty(max(nb, 1), dtype=torch.uint8, device=body.device)
    if ws is None:
        ws = workspace(nb, body.device)
    _require_gpu(plain, ok, ws)
    assert plain.numel() >= n and ok.numel() >= nb and ws.numel() >= _lib.lib().xs_workspace_bytes(nb)
    rc = _lib.lib().xs_open_object_dev(bytes(key), bytes(nonce0), first_block, body.data_ptr(), m,
                                       plain.data_ptr(), ok.data_ptr(), ws.data_ptr(), _stream(body))
    _lib.check(rc, "xs_open_object_dev")
    return plain[:n], ok[:nb]


def fill_random(t: torch.Tensor, seed: int):
    _require_gpu(t)
    rc = _lib.lib().xs_fill_random_dev(t.data_ptr(), t.numel() * t.element_size(), seed, _stream(t))
    _lib.check(rc, "xs_fill_random_dev")
    return t


def fill_blocks(t: torch.Tensor, first_block: int, block_stride: int, seed: int):
    """Fill t (whole 64 KiB blocks) with global blocks first_block + b*block_stride of the
    SplitMix64 stream that fill_random(seed) lays out contiguously."""
    _require_gpu(t)
    nbytes = t.numel() * t.element_size()
    if nbytes % BLOCK_DATA:
        raise ValueError("fill_blocks needs whole 64 KiB blocks")
    rc = _lib.lib().xs_fill_blocks_dev(t.data_ptr(), nbytes // BLOCK_DATA, first_block, block_stride, seed, _stream(t))
    _lib.check(rc, "xs_fill_blocks_dev")
    return t


def verify_blocks(t: torch.Tensor, first_block: int, block_stride: int, seed: int, mismatch: torch.Tensor):
    """Add to mismatch (one int64 on t's device) the number of 64-bit words of t (whole 64 KiB
    blocks) that differ from what fill_blocks(t, first_block, block_stride, seed) writes."""
    _require_gpu(t)
    nbytes = t.numel() * t.element_size()
    if nbytes % BLOCK_DATA:
        raise ValueError("verify_blocks needs whole 64 KiB blocks")
    if mismatch.dtype != torch.int64 or mismatch.numel() != 1 or mismatch.device != t.device:
        raise ValueError("verify_blocks: mismatch must be one int64 on the data's device")
    rc = _lib.lib().xs_verify_blocks_dev(t.data_ptr(), nbytes // BLOCK_DATA, first_block, block_stride, seed,
                                         ctypes_void(mismatch.data_ptr()), _stream(t))
    _lib.check(rc, "xs_verify_blocks_dev")


def _desc_tensor(desc, device):
    """xs_block_desc array (numpy structured, 48 B/entry, or a uint8 device tensor) on device."""
    if isinstance(desc, torch.Tensor):
        _require_gpu(desc)
        assert desc.numel() % 48 == 0
        return desc
    import numpy as np
    assert desc.dtype.itemsize == 48
    raw = np.frombuffer(desc.tobytes(), dtype=np.uint8)
    return torch.from_numpy(raw.copy()).to(device)


def seal_batch(key: bytes, desc, src: torch.Tensor, dst: torch.Tensor, ws: torch.Tensor = None):
    """Seal one secretbox per descriptor (xs_seal_batch_dev): src[src_off:+len] ->
    dst[dst_off:+16+len] with the descriptor's own nonce.  Invalid descriptors are skipped."""
    _require_gpu(src, dst)
    d = _desc_tensor(desc, src.device)
    nb = d.numel() // 48
    if ws is None:
        ws = workspace(nb, src.device)
    _require_gpu(ws)
    rc = _lib.lib().xs_seal_batch_dev(bytes(key), d.data_ptr(), nb, src.data_ptr(), src.numel(), dst.data_ptr(),
                                      dst.numel(), ws.data_ptr(), _stream(src))
    _lib.check(rc, "xs_seal_batch_dev")
    return dst


def open_batch(key: bytes, desc, src: torch.Tensor, dst: torch.Tensor, ok: torch.Tensor = None,
               ws: torch.Tensor = None) -> torch.Tensor:
    """Open one secretbox per descriptor (xs_open_batch_dev): src[src_off:+16+len] (tag||ct) ->
    dst[dst_off:+len]; returns ok (uint8 per descriptor; failed blocks are zero-filled,
    invalid descriptors write nothing and report 0)."""
    _require_gpu(src, dst)
    d = _desc_tensor(desc, src.device)
    nb = d.numel() // 48
    if ok is None:
        ok = torch.empty(max(nb, 1), dtype=torch.uint8, device=src.device)
    if ws is None:
        ws = workspace(nb, src.device)
    _require_gpu(ok, ws)
    rc = _lib.lib().xs_open_batch_dev(bytes(key), d.data_ptr(), nb, src.data_ptr(), src.numel(), dst.data_ptr(),
                                      dst.numel(), ok.data_ptr(), ws.data_ptr(), _stream(src))
    _lib.check(rc, "xs_open_batch_dev")
    return ok[:nb]


MD5_DESC_BYTES = 64


def md5_batch(desc, src: torch.Tensor):
    """MD5 of many streams in HBM (xs_md5_batch_dev): desc = numpy structured array of
    xs_md5_desc (off, len, prefix[32], prefix_len) or a uint8 device tensor; returns
    (digests uint8 [n,16], ok uint8 [n]) on the device."""
    _require_gpu(src)
    if isinstance(desc, torch.Tensor):
        _require_gpu(desc)
        d = desc
    else:
        import numpy as np
        assert desc.dtype.itemsize == MD5_DESC_BYTES
        d = torch.from_numpy(np.frombuffer(desc.tobytes(), dtype=np.uint8).copy()).to(src.device)
    n = d.numel() // MD5_DESC_BYTES
    dig = torch.empty(max(n, 1) * 16, dtype=torch.uint8, device=src.device)
    ok = torch.empty(max(n, 1), dtype=torch.uint8, device=src.device)
    rc = _lib.lib().xs_md5_batch_dev(d.data_ptr(), n, src.data_ptr(), src.numel(), dig.data_ptr(), ok.data_ptr(),
                                     _stream(src))
    _lib.check(rc, "xs_md5_batch_dev")
    return dig[:n * 16].view(-1, 16), ok[:n]
