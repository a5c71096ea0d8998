"""The HBG_ASYNC contract and device-mode argument checks (include/hbgpu.h,
"Conventions"; hydrabadger_amd/csrc/dev_err.h).

* A call made with HBG_DEVICE | HBG_ASYNC returns after enqueueing: the
  batched share verification (sort, batch sums, four group-testing rounds)
  reads its round counts on the device, so an encode and a verify enqueued
  back to back on one stream return while the stream is still busy and give
  the right bits after one hbg_sync.
* Device-mode index / length arguments are checked by the kernels: the
  offending item gets its invalid output and the next synchronisation point
  returns HBG_E_ARG (then clears it); nothing out of range is read.

Expected values come from construction (which shares were corrupted, which
index is out of range) and from the same call run on valid arguments.
"""
from __future__ import annotations

import struct

import numpy as np
import pytest

from oracle import bls12_381 as B
from oracle import tcrypto as T
from oracle import wire as owire
from tests import tdec_fixtures as fx


def _torch():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _ctx_on(torch, stream):
    from hydrabadger_amd import _lib
    ctx = _lib.Context(0)
    ctx.set_stream(stream.cuda_stream)
    return ctx


def _tdec_tables(torch, dev, sc):
    """Device tables of a fixture scenario: U, V, V_off, W, pk shares, all shares."""
    cts = sc["cts"]
    U = np.frombuffer(b"".join(B.g1_compress(c.U) for c in cts), np.uint8).copy()
    W = np.frombuffer(b"".join(B.g2_compress(c.W) for c in cts), np.uint8).copy()
    Vb = b"".join(bytes(c.V) for c in cts)
    off = np.zeros(len(cts) + 1, np.int64)
    off[1:] = np.cumsum([len(c.V) for c in cts])
    pk = np.frombuffer(b"".join(B.g1_compress(p) for p in sc["pk_shares"]), np.uint8).copy()
    n = len(sc["pk_shares"])
    sh = np.frombuffer(b"".join(B.g1_compress(sc["shares"][k][i]) for k in range(len(cts)) for i in range(n)),
                       np.uint8).copy()
    sct = np.repeat(np.arange(len(cts), dtype=np.int32), n)
    spk = np.tile(np.arange(n, dtype=np.int32), len(cts))
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    return d(U), d(np.frombuffer(Vb, np.uint8).copy()), d(off), d(W), d(pk), d(sh), d(sct), d(spk)


def _verify(ctx, tabs, n_ct, n_pk, sct, spk, ok, flags):
    from hydrabadger_amd import _lib
    U, V, off, W, pk, sh, _, _ = tabs
    return _lib.lib().hbg_tdec_verify_shares(ctx.h, n_ct, U.data_ptr(), V.data_ptr(), off.data_ptr(), W.data_ptr(),
                                             n_pk, pk.data_ptr(), ok.numel(), sh.data_ptr(), sct.data_ptr(),
                                             spk.data_ptr(), ok.data_ptr(), flags)


@pytest.mark.gpu
def test_async_encode_and_batched_verify_without_host_sync():
    torch = _torch()
    from hydrabadger_amd import _lib
    from hydrabadger_amd import broadcast as bc
    dev = torch.device("cuda:0")
    stream = torch.cuda.Stream(dev)
    ctx = _ctx_on(torch, stream)
    A = _lib.HBG_DEVICE | _lib.HBG_ASYNC
    # ~8 ms of RBC work ahead of the verify on the same stream
    n_nodes, P, B_ = 64, 1 << 20, 2048
    L = _lib.shard_len(n_nodes, P)
    S = (L + 15) // 16 * 16
    with torch.cuda.stream(stream):
        pay = torch.empty((B_, P), dtype=torch.uint8, device=dev)
        bc.synth_bytes(1, 0, P, pay, ctx=ctx, device=True)
        plen = torch.full((B_,), P, dtype=torch.int64, device=dev)
        shards = torch.empty((B_, n_nodes, S), dtype=torch.uint8, device=dev)
        levels = torch.empty((B_, _lib.merkle_nodes(n_nodes), 32), dtype=torch.uint8, device=dev)
        sc = fx.scenario(16, 6, 40, seed=11)
        tabs = _tdec_tables(torch, dev, sc)
        n_ct, n_pk = len(sc["cts"]), len(sc["pk_shares"])
        sct, spk = tabs[6].clone(), tabs[7].clone()
        bad = [3, 17, 40, 77]                        # claimed under another node's key
        for k in bad:
            spk[k] = (spk[k] + 1) % n_pk
        expect = np.ones(n_ct * n_pk, np.uint8)
        expect[bad] = 0
        ok = torch.zeros(n_ct * n_pk, dtype=torch.uint8, device=dev)

        def both():
            bc.rbc_encode_merkle_batch(n_nodes, pay, plen, L, shards, levels, ctx=ctx, device=True,
                                       asynchronous=True)
            _lib.check(_verify(ctx, tabs, n_ct, n_pk, sct, spk, ok, A), "verify")
        both()                                        # warm-up: grows every scratch slot once
        ctx.sync()
        ref_levels = levels.clone()
        ok.zero_()
        levels.zero_()
        stream.synchronize()
        both()
        busy = not stream.query()                     # the calls returned before the stream drained
        ctx.sync()
    assert busy, "an HBG_ASYNC call synchronised with the host"
    assert np.array_equal(ok.cpu().numpy(), expect)
    assert torch.equal(levels, ref_levels)


@pytest.mark.gpu
def test_device_mode_out_of_range_share_indices():
    torch = _torch()
    from hydrabadger_amd import _lib
    dev = torch.device("cuda:0")
    stream = torch.cuda.Stream(dev)
    ctx = _ctx_on(torch, stream)
    with torch.cuda.stream(stream):
        sc = fx.scenario(7, 3, 40, seed=5)
        tabs = _tdec_tables(torch, dev, sc)
        n_ct, n_pk = len(sc["cts"]), len(sc["pk_shares"])
        sct, spk = tabs[6].clone(), tabs[7].clone()
        sct[1] = n_ct            # ciphertext index out of range
        spk[9] = 1000            # key index out of range
        expect = np.ones(n_ct * n_pk, np.uint8)
        expect[[1, 9]] = 0
        for batched in (1, 3, 0):
            _lib.check(_lib.lib().hbg_test_set_tdec_batched(ctx.h, batched))
            ok = torch.full((n_ct * n_pk,), 7, dtype=torch.uint8, device=dev)
            # asynchronous: the call succeeds, the next synchronisation point reports it once
            assert _verify(ctx, tabs, n_ct, n_pk, sct, spk, ok, _lib.HBG_DEVICE | _lib.HBG_ASYNC) == 0
            assert _lib.lib().hbg_sync(ctx.h) == _lib.HBG_E_ARG
            assert _lib.lib().hbg_sync(ctx.h) == 0
            assert np.array_equal(ok.cpu().numpy(), expect), batched
            # synchronous device mode returns it directly
            ok.fill_(7)
            assert _verify(ctx, tabs, n_ct, n_pk, sct, spk, ok, _lib.HBG_DEVICE) == _lib.HBG_E_ARG
            assert np.array_equal(ok.cpu().numpy(), expect), batched
        _lib.check(_lib.lib().hbg_test_set_tdec_batched(ctx.h, 1))
        # host mode rejects the same arguments up front
        host = [t.cpu().numpy() for t in tabs]
        okh = np.zeros(n_ct * n_pk, np.uint8)
        sct_h = sct.cpu().numpy().view(np.uint32)
        spk_h = spk.cpu().numpy().view(np.uint32)
        rc = _lib.lib().hbg_tdec_verify_shares(ctx.h, n_ct, _lib.ptr(host[0]), _lib.ptr(host[1]), _lib.ptr(host[2]),
                                               _lib.ptr(host[3]), n_pk, _lib.ptr(host[4]), okh.size, _lib.ptr(host[5]),
                                               _lib.ptr(sct_h), _lib.ptr(spk_h), _lib.ptr(okh), 0)
        assert rc == _lib.HBG_E_ARG


@pytest.mark.gpu
def test_device_mode_sign_verify_decrypt_index_checks():
    torch = _torch()
    from hydrabadger_amd import _lib
    from hydrabadger_amd import threshold as th
    dev = torch.device("cuda:0")
    stream = torch.cuda.Stream(dev)
    ctx = _ctx_on(torch, stream)
    L = _lib.lib()
    D = _lib.HBG_DEVICE
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    sks = [12345, 67890, 1357911]
    sk = d(np.frombuffer(b"".join(th._scalar_bytes(k) for k in sks), np.uint8).copy())
    pk = d(np.frombuffer(b"".join(B.g1_compress(B.g1_mul(B.G1, k)) for k in sks), np.uint8).copy())
    msgs = [b"alpha", b"beta!", b"gamma"]
    mb = d(np.frombuffer(b"".join(msgs), np.uint8).copy())
    moff = d(np.array([0, 5, 10, 15], np.int64))
    with torch.cuda.stream(stream):
        who = d(np.array([0, 7, 2], np.int32))           # index 7 >= n_sk
        sig = torch.full((3, 96), 0x5A, dtype=torch.uint8, device=dev)
        assert L.hbg_bls_sign(ctx.h, 3, sk.data_ptr(), 3, who.data_ptr(), mb.data_ptr(), moff.data_ptr(),
                              sig.data_ptr(), D) == _lib.HBG_E_ARG
        s = sig.cpu().numpy()
        assert not s[1].any()
        assert s[0].tobytes() == B.g2_compress(T.sign(sks[0], msgs[0]))
        assert s[2].tobytes() == B.g2_compress(T.sign(sks[2], msgs[2]))
        ok = torch.full((3,), 9, dtype=torch.uint8, device=dev)
        good_sig = d(np.frombuffer(b"".join(B.g2_compress(T.sign(sks[i % 3], msgs[i])) for i in range(3)),
                                   np.uint8).copy())
        who_v = d(np.array([0, 1, 99], np.int32))        # index 99 >= n_pk
        assert L.hbg_bls_verify(ctx.h, 3, pk.data_ptr(), 3, who_v.data_ptr(), mb.data_ptr(), moff.data_ptr(),
                                good_sig.data_ptr(), ok.data_ptr(), D) == _lib.HBG_E_ARG
        assert ok.cpu().tolist() == [1, 1, 0]
        # decrypt_share_no_verify: (ct, sk) pairs with one of each out of range
        ct = T.encrypt(B.g1_mul(B.G1, 77), b"payload", 4242)
        U = d(np.frombuffer(B.g1_compress(ct.U), np.uint8).copy())
        sc_ = d(np.array([0, 1, 0], np.int32))
        ss_ = d(np.array([0, 0, 5], np.int32))
        share = torch.empty((3, 48), dtype=torch.uint8, device=dev)
        st = torch.empty(3, dtype=torch.int32, device=dev)
        assert L.hbg_tdec_decrypt_shares(ctx.h, 1, U.data_ptr(), 3, sk.data_ptr(), 3, sc_.data_ptr(), ss_.data_ptr(),
                                         share.data_ptr(), st.data_ptr(), D) == _lib.HBG_E_ARG
        assert st.cpu().tolist() == [0, _lib.HBG_E_ARG, _lib.HBG_E_ARG]
        assert share[0].cpu().numpy().tobytes() == B.g1_compress(T.decrypt_share(sks[0], ct))
        assert L.hbg_sync(ctx.h) == 0


@pytest.mark.gpu
def test_device_mode_encode_payload_length_check():
    torch = _torch()
    from hydrabadger_amd import _lib
    from hydrabadger_amd import broadcast as bc
    dev = torch.device("cuda:0")
    stream = torch.cuda.Stream(dev)
    ctx = _ctx_on(torch, stream)
    n_nodes, P, n = 16, 4096, 4
    L = _lib.shard_len(n_nodes, P)
    S = (L + 15) // 16 * 16
    with torch.cuda.stream(stream):
        pay = torch.zeros((n, P + 64), dtype=torch.uint8, device=dev)
        bc.synth_bytes(3, 0, P, pay, ctx=ctx, device=True)
        plen = torch.tensor([P, P + 100, P, 10 ** 9], dtype=torch.int64, device=dev)   # 1: wrong L, 3: > stride
        shards = torch.zeros((n, n_nodes, S), dtype=torch.uint8, device=dev)
        levels = torch.zeros((n, _lib.merkle_nodes(n_nodes), 32), dtype=torch.uint8, device=dev)
        bc.rbc_encode_merkle_batch(n_nodes, pay, plen, L, shards, levels, ctx=ctx, device=True, asynchronous=True)
        assert _lib.lib().hbg_sync(ctx.h) == _lib.HBG_E_ARG
        for k in (0, 2):
            ref_s, ref_t = bc.send_shards(pay[k, :P].cpu().numpy().tobytes(), n_nodes, ctx=ctx)
            assert np.array_equal(shards[k, :, :L].cpu().numpy(), ref_s)
            assert levels[k, -1].cpu().numpy().tobytes() == ref_t.root_hash()
        # a bad instance is skipped: its rows stay as they were
        assert not shards[1].any() and not shards[3].any()


@pytest.mark.gpu
def test_sig_combine_rejects_wrapping_threshold():
    from hydrabadger_amd import _lib
    ctx = _lib.default_context()
    sh = np.zeros(96, np.uint8)
    ix = np.zeros(1, np.uint32)
    out = np.zeros(96, np.uint8)
    par = np.zeros(1, np.uint8)
    st = np.zeros(1, np.int32)
    for t in (64, 0xFFFFFFFF):
        assert _lib.lib().hbg_sig_combine(ctx.h, t, 1, _lib.ptr(sh), _lib.ptr(ix), _lib.ptr(out), _lib.ptr(par),
                                          _lib.ptr(st), 0) == _lib.HBG_E_ARG


@pytest.mark.gpu
def test_frames_over_the_codec_limit():
    """LengthDelimitedCodec's 8 MiB max_frame_length: start_send refuses a
    longer frame (HBG_E_WIRE_FRAME), poll reports one as a framing error, and
    the largest legal frame still passes."""
    from hydrabadger_amd import _lib
    from hydrabadger_amd import wire as hw
    limit = owire.MAX_FRAME
    uid = struct.pack("<Q", 16) + bytes(range(16))                                  # Message(Uid, ..): a valid Uid
    big = struct.pack("<I", owire.KIND_MESSAGE) + uid + bytes(limit - 8 - 96 - 4 - 24 + 1)  # body = limit + 1
    with pytest.raises(_lib.HbgError) as e:
        hw.sign_frames([5], [(0, big)])
    assert e.value.code == _lib.HBG_E_WIRE_FRAME
    fits = big[:-1]                                                                 # body = limit
    (f_ok,) = hw.sign_frames([5], [(0, fits)])
    assert len(f_ok) == 4 + limit
    pk = B.g1_compress(B.g1_mul(B.G1, 5))
    over = struct.pack(">I", limit + 1) + f_ok[4:] + b"\0"
    st = hw.poll_frames([pk], [(0, f_ok), (0, over)])
    assert list(st) == [0, _lib.HBG_E_WIRE_FRAME]
    assert owire.poll_frame(over, B.g1_mul(B.G1, 5)) == owire.E_WIRE_FRAME


@pytest.mark.gpu
def test_device_mode_proof_msgs_index_check():
    torch = _torch()
    from hydrabadger_amd import _lib
    from hydrabadger_amd import broadcast as bc
    dev = torch.device("cuda:0")
    stream = torch.cuda.Stream(dev)
    ctx = _ctx_on(torch, stream)
    n_nodes, P, n = 8, 1000, 2
    L = _lib.shard_len(n_nodes, P)
    S = (L + 15) // 16 * 16
    with torch.cuda.stream(stream):
        pay = torch.zeros((n, 1008), dtype=torch.uint8, device=dev)
        bc.synth_bytes(4, 0, P, pay, ctx=ctx, device=True)
        plen = torch.full((n,), P, dtype=torch.int64, device=dev)
        shards = torch.zeros((n, n_nodes, S), dtype=torch.uint8, device=dev)
        levels = torch.zeros((n, _lib.merkle_nodes(n_nodes), 32), dtype=torch.uint8, device=dev)
        bc.rbc_encode_merkle_batch(n_nodes, pay, plen, L, shards, levels, ctx=ctx, device=True)
        idx = np.array([0, 3, 9, 5], np.uint32)          # leaf 9 >= N
        inst = np.array([0, 1, 1, 2], np.int64)           # instance 2 >= n
        off = bc.proof_msg_offsets(n_nodes, L, np.minimum(idx, n_nodes - 1))
        out = torch.full((int(off[-1]) + 16,), 0xEE, dtype=torch.uint8, device=dev)
        d = lambda a: torch.from_numpy(a).to(dev)  # noqa: E731
        rc = _lib.lib().hbg_rbc_write_proof_msgs(ctx.h, n_nodes, L, shards.data_ptr(), S, levels.data_ptr(), n,
                                                 _lib.HBG_MSG_VALUE, 4, d(inst).data_ptr(),
                                                 d(idx.view(np.int32)).data_ptr(), out.data_ptr(),
                                                 d(off.astype(np.int64)).data_ptr(), _lib.HBG_DEVICE)
        assert rc == _lib.HBG_E_ARG
        o = out.cpu().numpy()
        assert (o[int(off[2]):int(off[4])] == 0xEE).all()            # both bad messages unwritten
        assert o[int(off[0]):int(off[0]) + 4].tobytes() == struct.pack("<I", 0)


@pytest.mark.gpu
def test_oversized_tdec_batches_refused_before_anything_runs():
    """A batch larger than one grid (2^32 work-items) is HBG_E_ARG before any
    staging or launch: the outputs stay untouched and the context
    still works afterwards."""
    torch = _torch()
    from hydrabadger_amd import _lib
    dev = torch.device("cuda:0")
    stream = torch.cuda.Stream(dev)
    ctx = _ctx_on(torch, stream)
    with torch.cuda.stream(stream):
        pk = torch.zeros(48, dtype=torch.uint8, device=dev)
        r32 = torch.zeros(32, dtype=torch.uint8, device=dev)
        off = torch.zeros(2, dtype=torch.int64, device=dev)
        U = torch.full((48,), 0xAB, dtype=torch.uint8, device=dev)
        W = torch.full((96,), 0xCD, dtype=torch.uint8, device=dev)
        n = 1 << 32                                   # (n + 63) / 64 blocks x 64 > 2^32 - 1 work-items
        rc = _lib.lib().hbg_tdec_encrypt(ctx.h, pk.data_ptr(), n, r32.data_ptr(), r32.data_ptr(), off.data_ptr(),
                                         U.data_ptr(), U.data_ptr(), W.data_ptr(), _lib.HBG_DEVICE)
        assert rc == _lib.HBG_E_ARG
        sh = torch.zeros(48, dtype=torch.uint8, device=dev)
        ix = torch.zeros(1, dtype=torch.int32, device=dev)
        out = torch.full((16,), 0xEF, dtype=torch.uint8, device=dev)
        st = torch.full((1,), 7, dtype=torch.int32, device=dev)
        rc = _lib.lib().hbg_tdec_combine(ctx.h, 1, (1 << 26) + 1, sh.data_ptr(), ix.data_ptr(), out.data_ptr(),
                                         off.data_ptr(), out.data_ptr(), st.data_ptr(), _lib.HBG_DEVICE)
        assert rc == _lib.HBG_E_ARG
        torch.cuda.synchronize(dev)
        assert (U.cpu() == 0xAB).all() and (W.cpu() == 0xCD).all()
        assert (out.cpu() == 0xEF).all() and st.cpu().tolist() == [7]
        assert _lib.lib().hbg_sync(ctx.h) == 0
