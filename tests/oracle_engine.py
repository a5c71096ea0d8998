"""CPU stand-in for network.DeviceEngine built on the oracle (TEST
INFRASTRUCTURE: lets the product's epoch orchestration — hydrabadger_amd/
epoch.py, network.py — run under gloo without a GPU; never a product path).
Same method contract as DeviceEngine: CPU torch tensors in, CPU torch tensors
out."""
from __future__ import annotations

import numpy as np
import torch

from hydrabadger_amd import _lib, network
from oracle import bls12_381 as B
from oracle import corc, merkle as omerkle, tcrypto as T, wire


def _b(t) -> bytes:
    return t.contiguous().numpy().tobytes()


class OracleEngine:
    device = torch.device("cpu")

    def zeros(self, shape, dtype=torch.uint8):
        return torch.zeros(shape, dtype=dtype)

    def synth(self, tag, first, m, nbytes):
        return torch.from_numpy(np.stack([corc.synth_bytes(tag, first + k, nbytes) for k in range(m)]))

    def synth_payloads(self, first, m, P):
        from oracle import synth
        return self.synth(synth.TAG_PAYLOAD, first, m, P)

    def key_points(self, sk32):
        return torch.from_numpy(np.stack([np.frombuffer(B.g1_compress(B.g1_mul(B.G1, int.from_bytes(_b(r), "little"))),
                                                        np.uint8) for r in sk32]))

    def encrypt(self, pk48, msgs, r32):
        pk = B.g1_decompress(_b(pk48))
        U, V, W = [], [], []
        for k in range(msgs.shape[0]):
            ct = T.encrypt(pk, _b(msgs[k]), int.from_bytes(_b(r32[k]), "little"))
            U.append(np.frombuffer(B.g1_compress(ct.U), np.uint8))
            V.append(np.frombuffer(ct.V, np.uint8))
            W.append(np.frombuffer(B.g2_compress(ct.W), np.uint8))
        return (torch.from_numpy(np.stack(U)), torch.from_numpy(np.stack(V)).clone(),
                torch.from_numpy(np.stack(W)))

    def encode_merkle(self, N, pay, P):
        L = corc.shard_len(N, P)
        out = [corc.rbc_encode_merkle(N, pay[k, :P].numpy().copy()) for k in range(pay.shape[0])]
        return (torch.from_numpy(np.stack([s[:, :L] for s, _ in out])),
                torch.from_numpy(np.stack([lv for _, lv in out])))

    def write_proof_msgs(self, N, L, shards, levels, tag, inst, index, off):
        sib, nd = network.proof_index_map(N)
        sh, lv = shards.numpy(), levels.numpy()
        msgs = []
        for i, j in zip(inst.tolist(), index.tolist()):
            pr = omerkle.Proof(sh[i, j, :L].tobytes(), j, [lv[i, sib[j, q]].tobytes() for q in range(nd[j])],
                               lv[i, -1].tobytes())
            msgs.append(wire.serialize_proof_msg(tag, pr))
        buf = b"".join(msgs)
        assert len(buf) == int(off[-1])
        return torch.from_numpy(np.frombuffer(buf, np.uint8).copy())

    def read_msgs(self, N, L, buf, off):
        M = len(off) - 1
        S = (max(L, 1) + 15) // 16 * 16
        real_depth = _lib.merkle_depth(N)
        depth = max(real_depth, 1)
        tag, index, nd, st = (np.zeros(M, np.int64) for _ in range(4))
        vals, dig, roots = np.zeros((M, S), np.uint8), np.zeros((M, depth, 32), np.uint8), np.zeros((M, 32), np.uint8)
        raw = buf.numpy().tobytes()
        for q in range(M):
            s, tg, pl = wire.deserialize(raw[int(off[q]):int(off[q + 1])])
            st[q] = s
            tag[q] = tg if tg is not None else 0
            if s != wire.OK:
                continue
            if tg >= wire.READY:
                roots[q] = np.frombuffer(pl, np.uint8)
                continue
            index[q] = min(pl.index, 0xFFFFFFFF)
            roots[q] = np.frombuffer(pl.root_hash, np.uint8)
            k = len(pl.digests)
            if k > real_depth:  # more digests than any N-leaf proof: validate is false
                nd[q] = 0xFFFFFFFF
            else:
                nd[q] = k
                for d in range(k):
                    dig[q, d] = np.frombuffer(pl.digests[d], np.uint8)
            if len(pl.value) != L:
                st[q] = wire.E_INCORRECT_SHARD_SIZE
            else:
                vals[q, :L] = np.frombuffer(pl.value, np.uint8)
        i32 = lambda a: torch.from_numpy(a.astype(np.uint32).view(np.int32))
        return (i32(tag), torch.from_numpy(vals), i32(index), torch.from_numpy(dig), i32(nd), torch.from_numpy(roots),
                torch.from_numpy(st.astype(np.int32)))

    def validate_table(self, N, L, vals, index, dig, nd, roots, views=1):
        if views > 1:  # every view validates the table itself
            return torch.cat([self.validate_table(N, L, vals, index, dig, nd, roots) for _ in range(views)])
        ok = np.zeros(vals.shape[0], np.uint8)
        for q in range(vals.shape[0]):
            k = int(nd[q]) & 0xFFFFFFFF
            if k == 0xFFFFFFFF:
                continue
            pr = omerkle.Proof(vals[q, :L].numpy().tobytes(), int(index[q]) & 0xFFFFFFFF,
                               [dig[q, d].numpy().tobytes() for d in range(k)], roots[q].numpy().tobytes())
            ok[q] = pr.validate(N)
        return torch.from_numpy(ok)

    def decode(self, N, L, shards, present, roots, out=None):
        outs, lens, st = [], [], []
        for i in range(shards.shape[0]):
            r = None
            if int(present[i].sum()):
                r = corc.rbc_decode(N, L, shards[i].numpy().copy(), present[i].numpy(), roots[i].numpy().tobytes())
            outs.append(r or b"")
            lens.append(len(r) if r is not None else 0)
            st.append(1 if r is not None else 0)
        w = max([len(o) for o in outs] + [1])
        buf = np.zeros((len(outs), w), np.uint8)
        for i, o in enumerate(outs):
            buf[i, :len(o)] = np.frombuffer(o, np.uint8)
        if out is not None:  # the engine's in-place form (rows of a larger table)
            out[:, :w] = torch.from_numpy(buf)
            buf = out
        else:
            buf = torch.from_numpy(buf)
        return buf, torch.tensor(lens), torch.tensor(st, dtype=torch.uint8)

    def decrypt_shares(self, U48, sk32, pair_ct, pair_sk):
        Us = [B.g1_decompress(_b(u)) for u in U48]
        out = [np.frombuffer(B.g1_compress(T.decrypt_share(int.from_bytes(_b(sk32[s]), "little"), T.Ciphertext(
            Us[c], b"", None))), np.uint8) for c, s in zip(pair_ct.tolist(), pair_sk.tolist())]
        return torch.from_numpy(np.stack(out)) if out else torch.zeros((0, 48), dtype=torch.uint8)

    def threshold_decrypt(self, t, N, U, V, V_off, W, pk48, share48, arrival):
        k = U.shape[0]
        pks = [B.g1_decompress(_b(p)) for p in pk48]
        memo = {}   # one verdict memo per distinct (ciphertext, shares): the per-node views repeat them
        pt = np.zeros(max(int(V.numel()), 1), np.uint8)
        st = np.zeros(k, np.int32)
        oc = np.zeros((k, N), np.uint8)
        for q in range(k):
            v = _b(V[int(V_off[q]):int(V_off[q + 1])])
            try:
                ct = T.Ciphertext(B.g1_decompress(_b(U[q])), v, B.g2_decompress(_b(W[q])))
            except ValueError:
                st[q] = T.E_INVALID_CIPHERTEXT
                continue
            order = [int(s) & 0xFFFFFFFF for s in arrival[q].tolist()]  # u32 entries: markers, -1 ends
            shares = []
            for s in range(N):
                try:
                    shares.append(B.g1_decompress(_b(share48[q, s])))
                except ValueError:
                    shares.append(None)
            key = (_b(U[q]), v, _b(W[q]), _b(share48[q]))
            s_, p_, o_ = T.threshold_decrypt(t, ct, pks, shares, order, cache=memo.setdefault(key, {}))
            st[q] = s_
            oc[q] = o_
            if s_ == 0:
                pt[int(V_off[q]):int(V_off[q + 1])] = np.frombuffer(p_, np.uint8)
        return torch.from_numpy(pt[:int(V.numel())]), torch.from_numpy(st), torch.from_numpy(oc)

    def sync(self):
        pass
