//! Known answers for tests/golden/* from the real crates behind hydrabadger's
//! hot path (hbbft broadcast, threshold_crypto, bincode).  cargo is absent in
//! the build image, so this runs wherever cargo and the crates are:
//!
//!     cd rust/kat-gen && cargo run --release -- ../../tests/golden [--write]
//!
//! It recomputes with the crates, and compares byte for byte, every golden
//! value that does not depend on an RNG stream:
//!  * wire_golden.json trees: `Broadcast::broadcast(payload)` on an N-node
//!    `NetworkInfo` (hbbft's own send_shards: length prefix, padding,
//!    reed-solomon-erasure encode, Merkle tree over tiny-keccak SHA3-256), the
//!    N proofs bincode-serialised as `Message::Value` / `Message::Echo`, the
//!    root and `Message::Ready(root)`;
//!  * frames_golden.json: `SecretKey` from the fixture scalars, its public key
//!    and `sign(message)` bytes (f2, and hash_g2 through sign);
//!  * tdec_golden.json `hash_g2`: `SecretKey(1).sign(msg)` = hash_g2(msg) (a13);
//!  * tdec_golden.json scenario: the key polynomial -> `PublicKeySet` (its
//!    public key shares = the fixture's, which pins the share index
//!    convention), `Ciphertext::verify` of every fixture ciphertext,
//!    `verify_decryption_share` of every fixture share (and of each share
//!    claimed by the next node: false), `PublicKeySet::decrypt` of the first
//!    t+1 shares = the fixture plaintext (a12, a14, a15, a16); the bincode
//!    layout of `Ciphertext` / `DecryptionShare` that deserialises the
//!    fixture bytes is reported (version matrix row "ciphertext bytes");
//!  * bls_ops.json coin: `combine_signatures` of shares 1..=t+1 = the
//!    fixture signature, `Signature::parity` = the fixture parity (f3);
//!  * tdec_golden.json threshold_decrypt: hbbft's own `ThresholdDecrypt` of
//!    node 0 replays every case's `crate_arrival` (shares made by the crate
//!    on a generated network, the case's bad sender claiming another node's
//!    share) and must log exactly the fixture's faults per sender
//!    (MultipleDecryptionShares <-> the repeat flag,
//!    UnverifiedDecryptionShareSender <-> faulty) and output iff status 0
//!    (a18).
//! With `--write` the crate's values are also written to
//! `<golden dir>/crate_kat.json` (commit it with the Cargo.lock the run wrote:
//! together they are the version matrix DESIGN.md §3 asks for).  The exit
//! status is 0 iff every comparison matched; each mismatch is printed.
use std::collections::BTreeMap;
use std::convert::TryInto;
use std::fs;
use std::path::{Path, PathBuf};
use std::sync::Arc;

use hbbft::broadcast::{Broadcast, Message};
use hbbft::crypto::ff::PrimeField;
use hbbft::crypto::poly::Poly;
use hbbft::crypto::{Ciphertext, DecryptionShare, Fr, FrRepr, PublicKeySet, SecretKey, SecretKeySet,
                    SignatureShare};
use hbbft::threshold_decrypt::{FaultKind as TdFault, Message as TdMessage, ThresholdDecrypt};
use hbbft::NetworkInfo;
use serde::de::DeserializeOwned;
use serde::Serialize;
use serde_json::{json, Value};

// oracle/synth.py: the seeded payload generator the fixtures were made with
const BASE_SEED: u64 = 0x4842_4247;
const GAMMA: u64 = 0x9E37_79B9_7F4A_7C15;
const TAG_PAYLOAD: u64 = 1;

fn synth_bytes(tag: u64, instance: u64, n: usize) -> Vec<u8> {
    let s = BASE_SEED ^ (tag << 48) ^ instance;
    let mut out = Vec::with_capacity(n + 8);
    let mut k: u64 = 1;
    while out.len() < n {
        let mut z = s.wrapping_add(k.wrapping_mul(GAMMA));
        z = (z ^ (z >> 30)).wrapping_mul(0xBF58_476D_1CE4_E5B9);
        z = (z ^ (z >> 27)).wrapping_mul(0x94D0_49BB_1331_11EB);
        z ^= z >> 31;
        out.extend_from_slice(&z.to_le_bytes());
        k += 1;
    }
    out.truncate(n);
    out
}

#[derive(Default)]
struct Report {
    checked: usize,
    failed: usize,
    values: BTreeMap<String, String>,
}

impl Report {
    fn check(&mut self, what: String, got: &[u8], want_hex: &str) {
        let got_hex = hex::encode(got);
        self.checked += 1;
        if got_hex != want_hex {
            self.failed += 1;
            println!("MISMATCH {}\n  crate : {}\n  golden: {}", what, got_hex, want_hex);
        }
        self.values.insert(what, got_hex);
    }
}

fn load(dir: &Path, name: &str) -> Value {
    let text = fs::read_to_string(dir.join(name)).unwrap_or_else(|e| panic!("{}: {}", name, e));
    serde_json::from_str(&text).unwrap_or_else(|e| panic!("{}: {}", name, e))
}

fn hex_str(v: &Value) -> &str {
    v.as_str().expect("hex string")
}

fn check_wire(dir: &Path, rep: &mut Report) {
    let g = load(dir, "wire_golden.json");
    let mut rng = rand::thread_rng();
    for t in g["trees"].as_array().expect("trees") {
        let n = t["N"].as_u64().unwrap() as usize;
        let p = t["P"].as_u64().unwrap() as usize;
        let payload = synth_bytes(TAG_PAYLOAD, t["instance"].as_u64().unwrap(), p);
        // The keys do not enter the proofs: any NetworkInfo of N nodes will do.
        let infos: BTreeMap<usize, NetworkInfo<usize>> =
            NetworkInfo::generate_map(0..n, &mut rng).expect("NetworkInfo::generate_map");
        let mut bc = Broadcast::new(Arc::new(infos[&0].clone()), 0).expect("Broadcast::new");
        let step = bc.broadcast(payload).expect("Broadcast::broadcast");
        // Value(proof_i) to every other node, Echo(proof_0) from the proposer itself
        let mut proofs = BTreeMap::new();
        for tm in step.messages.iter() {
            match &tm.message {
                Message::Value(pr) | Message::Echo(pr) => {
                    proofs.insert(pr.index(), pr.clone());
                }
                _ => {}
            }
        }
        assert_eq!(proofs.len(), n, "N={}: one proof per node", n);
        let msgs = t["msgs"].as_array().expect("msgs");
        for (i, pr) in proofs.values().enumerate() {
            // the fixture alternates Value (even i) and Echo (odd i)
            let m = if i % 2 == 0 { Message::Value(pr.clone()) } else { Message::Echo(pr.clone()) };
            rep.check(format!("wire N={} P={} msg {}", n, p, i), &bincode::serialize(&m).unwrap(), hex_str(&msgs[i]));
        }
        let root = *proofs[&0].root_hash();
        rep.check(format!("wire N={} P={} root", n, p), &root, hex_str(&t["root"]));
        rep.check(format!("wire N={} P={} ready", n, p), &bincode::serialize(&Message::Ready(root)).unwrap(),
                  hex_str(&t["ready"]));
    }
}

/// A SecretKey from a 32-byte little-endian scalar (the fixtures' "sk" form).
fn secret_key(le_hex: &str) -> SecretKey {
    let b = hex::decode(le_hex).expect("sk hex");
    let mut limbs = [0u64; 4];
    for (i, l) in limbs.iter_mut().enumerate() {
        *l = u64::from_le_bytes(b[8 * i..8 * i + 8].try_into().unwrap());
    }
    let mut fr = Fr::from_repr(FrRepr(limbs)).expect("scalar < r");
    SecretKey::from_mut(&mut fr)
}

fn check_frames(dir: &Path, rep: &mut Report) {
    let g = load(dir, "frames_golden.json");
    let sks: Vec<SecretKey> = g["sk"].as_array().unwrap().iter().map(|s| secret_key(hex_str(s))).collect();
    for (i, sk) in sks.iter().enumerate() {
        rep.check(format!("frames pk {}", i), &sk.public_key().to_bytes(), hex_str(&g["pk"][i]));
    }
    for c in g["cases"].as_array().unwrap() {
        let m = hex::decode(hex_str(&c["message"])).unwrap();
        let s = c["signer"].as_u64().unwrap() as usize;
        rep.check(format!("frames sig {}", hex_str(&c["name"])), &sks[s].sign(&m).to_bytes(), hex_str(&c["sig"]));
    }
}

/// An Fr from a 32-byte little-endian scalar.
fn fr(le_hex: &str) -> Fr {
    let b = hex::decode(le_hex).expect("scalar hex");
    let mut limbs = [0u64; 4];
    for (i, l) in limbs.iter_mut().enumerate() {
        *l = u64::from_le_bytes(b[8 * i..8 * i + 8].try_into().unwrap());
    }
    Fr::from_repr(FrRepr(limbs)).expect("scalar < r")
}

/// Deserialises `T` from the first bincode layout among `forms` that both
/// parses and re-serialises to the same bytes; returns the value and the
/// layout's index (point tuples vs length-prefixed byte strings differ
/// between threshold_crypto versions).
fn de_any<T: DeserializeOwned + Serialize>(forms: &[Vec<u8>]) -> Option<(T, usize)> {
    forms.iter().enumerate().find_map(|(i, f)| {
        let v: T = bincode::deserialize(f).ok()?;
        if bincode::serialize(&v).ok()? == *f { Some((v, i)) } else { None }
    })
}

fn len_prefixed(b: &[u8]) -> Vec<u8> {
    let mut v = (b.len() as u64).to_le_bytes().to_vec();
    v.extend_from_slice(b);
    v
}

/// The two candidate bincode layouts of a compressed point.
fn point_forms(b: &[u8]) -> Vec<Vec<u8>> {
    vec![b.to_vec(), len_prefixed(b)]
}

/// `Ciphertext(U, V, W)` from the fixture's compressed U, V and compressed W.
fn ciphertext(u: &[u8], v: &[u8], w: &[u8]) -> (Ciphertext, usize) {
    let forms: Vec<Vec<u8>> = (0..2)
        .map(|i| {
            let mut f = point_forms(u)[i].clone();
            f.extend_from_slice(&len_prefixed(v));
            f.extend_from_slice(&point_forms(w)[i]);
            f
        })
        .collect();
    de_any::<Ciphertext>(&forms).expect("no bincode layout of Ciphertext parses the fixture bytes")
}

fn decryption_share(b: &[u8]) -> DecryptionShare {
    de_any::<DecryptionShare>(&point_forms(b)).expect("DecryptionShare layout").0
}

fn bits(b: bool) -> Vec<u8> {
    vec![b as u8]
}

fn check_tdec(dir: &Path, rep: &mut Report) {
    let g = load(dir, "tdec_golden.json");
    let sc = &g["scenario"];
    let t = sc["t"].as_u64().unwrap() as usize;
    let poly = Poly::from(sc["poly"].as_array().unwrap().iter().map(|c| fr(hex_str(c))).collect::<Vec<Fr>>());
    let sks = SecretKeySet::from(poly);
    let pks: PublicKeySet = sks.public_keys();
    assert_eq!(pks.threshold(), t, "poly degree");
    for (i, p) in sc["pk_shares"].as_array().unwrap().iter().enumerate() {
        rep.check(format!("tdec pk_share {}", i), &pks.public_key_share(i).to_bytes(), hex_str(p));
    }
    for (k, c) in sc["cts"].as_array().unwrap().iter().enumerate() {
        let (ct, layout) = ciphertext(&hex::decode(hex_str(&c["U"])).unwrap(), &hex::decode(hex_str(&c["V"])).unwrap(),
                                      &hex::decode(hex_str(&c["W"])).unwrap());
        rep.values.insert(format!("tdec ct {} bincode layout", k),
                          (if layout == 0 { "point tuples" } else { "length-prefixed points" }).to_string());
        rep.check(format!("tdec ct {} verify", k), &bits(ct.verify()), "01");
        let shares: Vec<DecryptionShare> = c["shares"].as_array().unwrap().iter()
            .map(|x| decryption_share(&hex::decode(hex_str(x)).unwrap())).collect();
        let n = shares.len();
        for (i, sh) in shares.iter().enumerate() {
            rep.check(format!("tdec ct {} share {} verify", k, i),
                      &bits(pks.public_key_share(i).verify_decryption_share(sh, &ct)), "01");
            // the same bytes claimed by the next node
            rep.check(format!("tdec ct {} share {} as node {} verify", k, i, (i + 1) % n),
                      &bits(pks.public_key_share((i + 1) % n).verify_decryption_share(sh, &ct)), "00");
            // and the crate's own share of node i is the fixture's
            let own = sks.secret_key_share(i).decrypt_share_no_verify(&ct);
            rep.check(format!("tdec ct {} share {} bytes", k, i), &bincode::serialize(&own).unwrap()
                          [bincode::serialize(&own).unwrap().len() - 48..], hex_str(&c["shares"][i]));
        }
        let pt = pks.decrypt((0..=t).map(|i| (i, &shares[i])), &ct).expect("PublicKeySet::decrypt");
        rep.check(format!("tdec ct {} decrypt", k), &pt, hex_str(&c["plaintext"]));
    }
}

fn check_coin(dir: &Path, rep: &mut Report) {
    let g = load(dir, "bls_ops.json");
    let c = &g["coin"];
    let t = c["t"].as_u64().unwrap() as usize;
    // the coin uses the tdec scenario's key set (tests/golden/make_golden_bls.py)
    let sc = load(dir, "tdec_golden.json");
    let poly = Poly::from(sc["scenario"]["poly"].as_array().unwrap().iter().map(|x| fr(hex_str(x)))
                              .collect::<Vec<Fr>>());
    let pks = SecretKeySet::from(poly).public_keys();
    rep.check("coin pk".to_string(), &pks.public_key().to_bytes(), hex_str(&c["pk"]));
    for (j, coin) in c["coins"].as_array().unwrap().iter().enumerate() {
        let shares: Vec<SignatureShare> = coin["shares"].as_array().unwrap().iter()
            .map(|x| de_any::<SignatureShare>(&point_forms(&hex::decode(hex_str(x)).unwrap()))
                 .expect("SignatureShare layout").0)
            .collect();
        let doc = hex::decode(hex_str(&coin["doc"])).unwrap();
        for (i, sh) in shares.iter().enumerate() {
            rep.check(format!("coin {} share {} verify", j, i), &bits(pks.public_key_share(i).verify(sh, &doc)), "01");
        }
        let sig = pks.combine_signatures((1..=t + 1).map(|i| (i, &shares[i]))).expect("combine_signatures");
        rep.check(format!("coin {} sig", j), &sig.to_bytes(), hex_str(&coin["sig"]));
        let want = if coin["parity"].as_bool().unwrap() { "01" } else { "00" };
        rep.check(format!("coin {} parity", j), &bits(sig.parity()), want);
    }
}

fn check_threshold_decrypt(dir: &Path, rep: &mut Report) {
    let g = load(dir, "tdec_golden.json");
    let sc = &g["scenario"];
    let a = &g["threshold_decrypt"];
    let n = sc["pk_shares"].as_array().unwrap().len();
    let our = a["our_node"].as_u64().unwrap() as usize;
    let rf = a["outcome_codes"]["repeat_flag"].as_u64().unwrap() as u8;
    let faulty = a["outcome_codes"]["faulty"].as_u64().unwrap() as u8;
    let mut rng = rand::thread_rng();
    let infos: BTreeMap<usize, NetworkInfo<usize>> =
        NetworkInfo::generate_map(0..n, &mut rng).expect("NetworkInfo::generate_map");
    for (ci, c) in a["cases"].as_array().unwrap().iter().enumerate() {
        let k = c["ct"].as_u64().unwrap() as usize;
        let msg = hex::decode(hex_str(&sc["cts"][k]["plaintext"])).unwrap();
        let ct = infos[&our].public_key_set().public_key().encrypt(&msg);
        let mut shares: Vec<DecryptionShare> = (0..n)
            .map(|i| infos[&i].secret_key_share().expect("validator").decrypt_share_no_verify(&ct))
            .collect();
        let bad = c["bad_sender"].as_u64().unwrap() as usize;
        shares[bad] = shares[(bad + 1) % n].clone();
        let mut td = ThresholdDecrypt::new(Arc::new(infos[&our].clone()));
        let mut faults: BTreeMap<usize, Vec<String>> = BTreeMap::new();
        let mut output: Option<Vec<u8>> = None;
        let mut absorb = |step: hbbft::threshold_decrypt::Step<usize>| {
            for f in step.fault_log.0.iter() {
                faults.entry(f.node_id).or_default().push(format!("{:?}", f.kind));
            }
            if let Some(o) = step.output.into_iter().next() {
                output = Some(o);
            }
        };
        let arr = c["crate_arrival"].as_array().unwrap();
        let start = |td: &mut ThresholdDecrypt<usize>| {
            td.set_ciphertext(ct.clone()).expect("set_ciphertext");
            td.start_decryption().expect("start_decryption")
        };
        if !arr.iter().any(|x| x.is_string()) {
            absorb(start(&mut td));
        }
        for x in arr {
            if x.is_string() {
                absorb(start(&mut td));
            } else {
                let s = x.as_u64().unwrap() as usize;
                absorb(td.handle_message(&s, TdMessage(shares[s].clone())).expect("handle_message"));
            }
        }
        let oc = c["outcome"].as_array().unwrap();
        for (s, o) in oc.iter().enumerate() {
            let o = o.as_u64().unwrap() as u8;
            let got = faults.get(&s).cloned().unwrap_or_default();
            let want_repeat = o & rf != 0;
            let want_unverified = o & 3 == faulty;
            let has = |kind: TdFault| got.iter().any(|g| *g == format!("{:?}", kind));
            let ok = has(TdFault::MultipleDecryptionShares) == want_repeat
                && has(TdFault::UnverifiedDecryptionShareSender) == want_unverified;
            rep.check(format!("a18 case {} sender {} faults", ci, s), &bits(ok), "01");
        }
        let status = c["status"].as_i64().unwrap();
        rep.check(format!("a18 case {} output", ci), &bits(output.is_some()), if status == 0 { "01" } else { "00" });
        if let Some(o) = output {
            rep.check(format!("a18 case {} plaintext", ci), &o, &hex::encode(&msg));
        }
    }
}

fn check_hash_g2(dir: &Path, rep: &mut Report) {
    let g = load(dir, "tdec_golden.json");
    let one = secret_key(&format!("01{}", "00".repeat(31)));
    for h in g["hash_g2"].as_array().unwrap() {
        let m = hex::decode(hex_str(&h["msg"])).unwrap();
        rep.check(format!("hash_g2 msg={}", hex_str(&h["msg"])), &one.sign(&m).to_bytes(), hex_str(&h["point"]));
    }
}

fn main() {
    let args: Vec<String> = std::env::args().skip(1).collect();
    let write = args.iter().any(|a| a == "--write");
    let dir = args.iter().find(|a| !a.starts_with("--")).map(PathBuf::from)
        .unwrap_or_else(|| PathBuf::from("../../tests/golden"));
    let mut rep = Report::default();
    check_wire(&dir, &mut rep);
    check_frames(&dir, &mut rep);
    check_hash_g2(&dir, &mut rep);
    check_tdec(&dir, &mut rep);
    check_coin(&dir, &mut rep);
    check_threshold_decrypt(&dir, &mut rep);
    println!("kat-gen: {} comparisons, {} mismatches", rep.checked, rep.failed);
    if write {
        let out = json!({"generator": "rust/kat-gen", "values": rep.values});
        fs::write(dir.join("crate_kat.json"), serde_json::to_string_pretty(&out).unwrap()).expect("write");
    }
    std::process::exit(if rep.failed == 0 { 0 } else { 1 });
}
