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
//!  * tdec_golden.json `hash_g2`: `SecretKey(1).sign(msg)` = hash_g2(msg) (a13).
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
use hbbft::crypto::{Fr, FrRepr, SecretKey};
use hbbft::NetworkInfo;
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
    println!("kat-gen: {} comparisons, {} mismatches", rep.checked, rep.failed);
    if write {
        let out = json!({"generator": "rust/kat-gen", "values": rep.values});
        fs::write(dir.join("crate_kat.json"), serde_json::to_string_pretty(&out).unwrap()).expect("write");
    }
    std::process::exit(if rep.failed == 0 { 0 } else { 1 });
}
