//! Safe wrappers over the raw FFI with the argument meaning and errors of the
//! hbbft / threshold_crypto surfaces they replace, for the
//! patch points listed in INTEGRATION.md §4.  Host buffers (no HBG_DEVICE):
//! the engine stages them through device memory.
use super::*;
use std::ffi::CStr;
use std::sync::Mutex;

/// An engine error: the negative `HBG_E_*` code and its name
/// (`hbg_strerror`, which mirrors the rse / threshold_crypto variant names).
#[derive(Debug, Clone, PartialEq, Eq)]
pub struct Error {
    pub code: i32,
}

impl std::fmt::Display for Error {
    fn fmt(&self, f: &mut std::fmt::Formatter<'_>) -> std::fmt::Result {
        let name = unsafe { CStr::from_ptr(hbg_strerror(self.code)) };
        write!(f, "{} ({})", name.to_string_lossy(), self.code)
    }
}

impl std::error::Error for Error {}

fn check(rc: c_int) -> Result<(), Error> {
    if rc == HBG_OK {
        Ok(())
    } else {
        Err(Error { code: rc })
    }
}

/// One device context (one GPU, one stream).  hydrabadger runs its
/// consensus on one tokio worker under the state lock (SURVEY.md §8(b)
/// "threading: sync"); the mutex serialises the rare concurrent caller.
pub struct Engine {
    ctx: Mutex<*mut hbg_ctx>,
}

unsafe impl Send for Engine {}
unsafe impl Sync for Engine {}

impl Engine {
    pub fn new(device: i32) -> Result<Engine, Error> {
        let mut ctx: *mut hbg_ctx = std::ptr::null_mut();
        check(unsafe { hbg_init(&mut ctx, device) })?;
        Ok(Engine { ctx: Mutex::new(ctx) })
    }

    /// Share-verification schedule (`hbg_set_share_verify`): `per_share =
    /// true` makes every decryption / coin share bit the crate's own
    /// per-share pairing equation (deterministic); the default batched
    /// schedule differs from it with probability <= 2^-127 per check.
    pub fn set_share_verify_per_share(&self, per_share: bool) -> Result<(), Error> {
        let mode = if per_share { HBG_VERIFY_PER_SHARE } else { HBG_VERIFY_BATCHED };
        self.with(|c| check(unsafe { hbg_set_share_verify(c, mode) }))
    }

    fn with<R>(&self, f: impl FnOnce(*mut hbg_ctx) -> R) -> R {
        let g = self.ctx.lock().unwrap();
        f(*g)
    }

    /// `Coding::encode(&mut [&mut [u8]])` for the Reed-Solomon variant:
    /// parity rows are rewritten in place from the data rows.
    pub fn coding_encode(&self, data: usize, parity: usize, slices: &mut [&mut [u8]]) -> Result<(), Error> {
        let n = data + parity;
        if slices.len() != n {
            return Err(Error { code: HBG_E_TOO_FEW_SHARDS });
        }
        let l = slices[0].len();
        if slices.iter().any(|s| s.len() != l) {
            return Err(Error { code: HBG_E_INCORRECT_SHARD_SIZE });
        }
        // send_shards' buffer is one contiguous N*L allocation chunked with
        // chunks_mut(L): pass it in place; other layouts are gathered.
        let base = slices[0].as_mut_ptr();
        let contiguous = slices.iter().enumerate().all(|(i, s)| s.as_ptr() as usize == base as usize + i * l);
        if contiguous {
            return self.with(|c| check(unsafe {
                hbg_rs_encode(c, data as u32, parity as u32, l as u64, base, l as u64, 1, 0)
            }));
        }
        let mut buf = vec![0u8; n * l];
        for (i, s) in slices.iter().enumerate() {
            buf[i * l..(i + 1) * l].copy_from_slice(s);
        }
        self.with(|c| check(unsafe {
            hbg_rs_encode(c, data as u32, parity as u32, l as u64, buf.as_mut_ptr(), l as u64, 1, 0)
        }))?;
        for (i, s) in slices.iter_mut().enumerate().skip(data) {
            s.copy_from_slice(&buf[i * l..(i + 1) * l]);
        }
        Ok(())
    }

    /// `Coding::reconstruct_shards(&mut [Option<Box<[u8]>>])`: the `None`
    /// slots are filled from the first `data` present rows; present rows are
    /// left as received; fewer than `data` present -> TooFewShardsPresent.
    pub fn reconstruct_shards(&self, data: usize, parity: usize, shards: &mut [Option<Box<[u8]>>])
                              -> Result<(), Error> {
        let n = data + parity;
        if shards.len() != n {
            return Err(Error { code: HBG_E_TOO_FEW_SHARDS });
        }
        let l = match shards.iter().flatten().next() {
            Some(s) => s.len(),
            None => return Err(Error { code: HBG_E_TOO_FEW_SHARDS_PRESENT }),
        };
        if shards.iter().flatten().any(|s| s.len() != l) {
            return Err(Error { code: HBG_E_INCORRECT_SHARD_SIZE });
        }
        if l == 0 {
            return Err(Error { code: HBG_E_EMPTY_SHARD });
        }
        if shards.iter().all(|s| s.is_some()) {
            return Ok(());
        }
        // gather: one N*L buffer + present[N]
        let mut buf = vec![0u8; n * l];
        let mut present = vec![0u8; n];
        for (i, s) in shards.iter().enumerate() {
            if let Some(s) = s {
                buf[i * l..(i + 1) * l].copy_from_slice(s);
                present[i] = 1;
            }
        }
        let mut status = 0i32;
        self.with(|c| check(unsafe {
            hbg_rs_reconstruct(c, data as u32, parity as u32, l as u64, buf.as_mut_ptr(), l as u64,
                               present.as_ptr(), &mut status, 1, 0)
        }))?;
        check(status)?;
        // scatter: new boxes for the None slots
        for (i, s) in shards.iter_mut().enumerate() {
            if s.is_none() {
                *s = Some(buf[i * l..(i + 1) * l].to_vec().into_boxed_slice());
            }
        }
        Ok(())
    }

    /// `MerkleTree::from_vec(values)`: the flat `levels` digests, root last.
    pub fn merkle_levels(&self, values: &[Vec<u8>]) -> Result<Vec<[u8; 32]>, Error> {
        let n = values.len();
        let l = values.first().map(|v| v.len()).unwrap_or(0);
        if values.iter().any(|v| v.len() != l) {
            return Err(Error { code: HBG_E_INCORRECT_SHARD_SIZE });
        }
        let mut buf = Vec::with_capacity(n * l);
        for v in values {
            buf.extend_from_slice(v);
        }
        let nodes = unsafe { hbg_merkle_nodes(n as u32) } as usize;
        let mut levels = vec![[0u8; 32]; nodes];
        self.with(|c| check(unsafe {
            hbg_merkle_build(c, n as u32, l as u64, buf.as_ptr(), l as u64, levels.as_mut_ptr() as *mut u8, 1, 0)
        }))?;
        Ok(levels)
    }

    /// `Proof::validate(n)` for one proof.
    pub fn proof_validate(&self, n: u32, value: &[u8], index: u32, digests: &[[u8; 32]], root: &[u8; 32])
                          -> Result<bool, Error> {
        let depth = unsafe { hbg_merkle_depth(n) } as usize;
        if digests.len() > depth {
            return Ok(false); // more digests than any n-leaf proof
        }
        let mut dig = vec![[0u8; 32]; depth.max(1)];
        dig[..digests.len()].copy_from_slice(digests);
        let nd = digests.len() as u32;
        let mut ok = 0u8;
        self.with(|c| check(unsafe {
            hbg_merkle_validate(c, n, value.len() as u64, value.as_ptr(), value.len() as u64, &index,
                                dig.as_ptr() as *const u8, &nd, root.as_ptr(), &mut ok, 1, 0)
        }))?;
        Ok(ok == 1)
    }

    /// hbbft ThresholdDecrypt for an epoch (hbg_tdec_threshold_decrypt):
    /// `cts[k] = (U48, V, W96)`, `shares[k][i]` = sender i's share of ct k
    /// (None: never arrived), `arrival[k]` = sender order, repeats allowed,
    /// with `HBG_ARRIVAL_CIPHERTEXT` where the ciphertext arrives at an
    /// observer, or `HBG_ARRIVAL_OWN | i` where it arrives at validator node i
    /// (its own share is inserted before try_output) (None: node order,
    /// after the ciphertext).  Returns per ciphertext `Ok(plaintext)`
    /// or the status code, and the per-sender outcomes (HBG_SHARE_*, possibly
    /// | HBG_SHARE_REPEAT).
    #[allow(clippy::type_complexity)]
    pub fn threshold_decrypt(&self, t: u32, pk_shares: &[[u8; 48]], cts: &[([u8; 48], Vec<u8>, [u8; 96])],
                             shares: &[Vec<Option<[u8; 48]>>], arrival: Option<&[Vec<u32>]>)
                             -> Result<(Vec<Result<Vec<u8>, Error>>, Vec<Vec<u8>>), Error> {
        let n_ct = cts.len();
        let n = pk_shares.len();
        let mut u = Vec::with_capacity(48 * n_ct);
        let mut w = Vec::with_capacity(96 * n_ct);
        let mut v = Vec::new();
        let mut off = vec![0u64; n_ct + 1];
        for (k, (uu, vv, ww)) in cts.iter().enumerate() {
            u.extend_from_slice(uu);
            w.extend_from_slice(ww);
            v.extend_from_slice(vv);
            off[k + 1] = v.len() as u64;
        }
        let mut sh = vec![0u8; 48 * n * n_ct];
        // the arrivals that reach the instance (senders that sent a share, and the marker)
        let mut sent: Vec<Vec<u32>> = Vec::with_capacity(n_ct);
        for k in 0..n_ct {
            let order: Vec<u32> = match arrival {
                Some(a) => a[k].clone(),
                None => (0..n as u32).collect(),
            };
            for (i, x) in shares[k].iter().enumerate() {
                if let Some(x) = x {
                    sh[48 * (k * n + i)..48 * (k * n + i + 1)].copy_from_slice(x);
                }
            }
            let marker = |s: u32| s == HBG_ARRIVAL_CIPHERTEXT
                || (s & HBG_ARRIVAL_OWN != 0 && ((s & !HBG_ARRIVAL_OWN) as usize) < n);
            // an entry >= n that is no marker ends the list
            sent.push(order.into_iter()
                .take_while(|&s| marker(s) || (s as usize) < n)
                .filter(|&s| marker(s) || shares[k][s as usize].is_some())
                .collect());
        }
        let alen = sent.iter().map(|o| o.len() + 1).max().unwrap_or(1);
        let mut arr = vec![u32::MAX; alen * n_ct];
        for (k, o) in sent.iter().enumerate() {
            arr[k * alen..k * alen + o.len()].copy_from_slice(o);
        }
        let pk: Vec<u8> = pk_shares.iter().flat_map(|p| p.iter().copied()).collect();
        let mut pt = vec![0u8; v.len().max(1)];
        let mut status = vec![0i32; n_ct];
        let mut outcome = vec![0u8; n * n_ct];
        self.with(|c| check(unsafe {
            hbg_tdec_threshold_decrypt(c, t, n as u32, n_ct as u32, u.as_ptr(), v.as_ptr(), off.as_ptr(),
                                       w.as_ptr(), pk.as_ptr(), sh.as_ptr(), arr.as_ptr(), alen as u32,
                                       pt.as_mut_ptr(), status.as_mut_ptr(), outcome.as_mut_ptr(), 0)
        }))?;
        let out = (0..n_ct)
            .map(|k| if status[k] == 0 {
                Ok(pt[off[k] as usize..off[k + 1] as usize].to_vec())
            } else {
                Err(Error { code: status[k] })
            })
            .collect();
        Ok((out, outcome.chunks(n).map(|c| c.to_vec()).collect()))
    }
}

impl Drop for Engine {
    fn drop(&mut self) {
        let c = *self.ctx.lock().unwrap();
        unsafe { hbg_free(c) };
    }
}
