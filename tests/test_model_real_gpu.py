"""Parity at the pinned checkpoints' real shapes (qwen3-asr-0.6b / qwen3-asr-1.7b, hf_cache_utils.py:11-26;
called through transcribe_cpp.Model(...).session(...).run(...), qwen3_asr_server.py:122-123,321).

The GGUF weights are not provisioned here, so both sides take the seeded synthetic weights with the exact tensor
shapes (the GPU generator and the oracle's are bit-identical: first test).  Then, through the C ABI and at the
real dimensions — 18/24 encoder layers with 104-token attention windows, 28 decoder layers, GQA 16/8, the
151,936-row tied vocabulary projection, the K = 3,072/6,144 down projections:

  * log-mel and the encoder / projector outputs against the oracle;
  * prefill logits (the MFMA GEMM + tile attention path) and teacher-forced decode logits (the GEMV path);
  * greedy tokens equal to the oracle's up to the first near-tie;
  * (1.7B) an 8-segment batch (MFMA decode GEMMs, continuous batching, step graphs) token-equal to the single
    runs and to the oracle, and the MXFP8 precision mode against the Q8 path.

Both sides compute the same W8A8 Q8_0 / f16-KV semantics and differ only in f32 summation order, so the bounds
are relative errors set at about 2x the errors observed on MI355X (observed values in each test's comment;
$QASR_PARITY_LOG collects them).
"""
import numpy as np
import pytest

import oracle
from bench import speech_like
from conftest import record

pytestmark = pytest.mark.gpu

SEED = 7
ARCHS = ["qwen3-asr-0.6b", "qwen3-asr-1.7b"]
SP = oracle.QWEN_SPECIAL


def rel_err(a, b):
    return float(np.abs(a - b).max() / (np.abs(b).max() + 1e-12))


def clip(seconds, seed):
    return speech_like(np.random.default_rng(seed), int(seconds * 16000))


@pytest.fixture(scope="module", params=ARCHS)
def pair(request, torch_dev):
    from qasr.transcribe_cpp import Model

    arch = request.param
    m = Model.synthetic(arch, seed=SEED)
    s = m.session(kv_type="f16", n_ctx=4096)
    oracle.set_mode(engine=True)
    o = oracle.Model(oracle.arch_config(arch), seed=SEED)
    yield arch, m, s, o
    s.close()
    m.close()


def _near_tie(lg_row, frac=0.005):
    """top-2 gap below 0.5 % of the row's range (r3: the synthetic vocabulary's log-normal row norms give ≥ 90 % of
    decode rows a clear margin; r2 used 2 % of max|logit| on i.i.d. rows)"""
    top2 = np.sort(lg_row)[-2:]
    return top2[1] - top2[0] < frac * (lg_row.max() - lg_row.min())


def test_real_shapes_synthetic_weights_bit_exact(pair):
    """the device generator and the oracle's agree bit for bit on tensors of every kind at the real shapes"""
    arch, m, _, o = pair
    hp = m.hparams
    assert {k: hp[k] for k in oracle.CFG_INT_KEYS} == {k: o.cfg[k] for k in oracle.CFG_INT_KEYS}
    last = hp["txt_layers"] - 1
    for name in ["a.conv2.weight", "a.conv_out.weight", "a.blk.0.attn_q.bias", f"a.blk.{hp['enc_layers'] - 1}.ffn_down.weight",
                 "a.proj2.weight", "blk.0.attn_k.weight", "blk.0.ffn_gate.weight", f"blk.{last}.ffn_up.weight",
                 f"blk.{last}.ffn_down.weight", f"blk.{last}.attn_q_norm.weight", "output_norm.weight"]:
        ref = o.export_one(name)
        got = m.export_tensor(name, ref.nbytes)
        assert np.array_equal(got, ref), name


def test_real_mel_and_encoder(pair):
    """9 s of speech-like audio: 900 mel frames → 117 audio tokens in two attention windows (104 + 13)"""
    arch, _, s, o = pair
    audio = clip(9.0, 11)
    mel, tv = s.mel(audio)
    rmel, rtv = oracle.mel(audio)
    assert tv == rtv == 900
    mel_err = float(np.abs(mel - rmel).max())
    emb, enc = s.encode(rmel, rtv, want_enc=True)
    remb, renc = o.encode(rmel, rtv, want_enc=True)
    assert emb.shape == remb.shape == (117, o.cfg["txt_h"])
    e_enc, e_emb = rel_err(enc, renc), rel_err(emb, remb)
    record(f"real_encoder[{arch}]", mel_abs=mel_err, enc_rel=e_enc, emb_rel=e_emb)
    # observed on MI355X (r2): mel 2.6e-5 abs; enc 1.02e-2 / 1.05e-2, emb 1.64e-2 / 1.76e-2 rel (0.6B / 1.7B)
    assert mel_err < 5e-5
    assert e_enc < 2e-2 and e_emb < 3.5e-2


def _prompt_embeds(o, audio):
    rmel, rtv = oracle.mel(audio)
    remb = o.encode(rmel, rtv)
    ids = np.array(oracle.chat_prompt(remb.shape[0]), np.int32)
    return ids, remb


def test_real_prefill_logits(pair):
    """the whole prompt through the prefill path (MFMA Q8 GEMMs, tile attention, shared-weight lm_head)"""
    arch, _, s, o = pair
    ids, remb = _prompt_embeds(o, clip(2.5, 12))
    kv = oracle.KV(o, 256)
    x = kv.embed(ids)
    x[ids == SP["tok_audio_pad"]] = remb
    ref = kv.forward(x, all_logits=True)
    got = s.prefill_logits(x)
    e = rel_err(got, ref)
    agree = float((got.argmax(1) == ref.argmax(1)).mean())
    clear = np.array([not _near_tie(r) for r in ref])
    record(f"real_prefill_logits[{arch}]", logits_rel=e, argmax_agree=agree, rows=len(ids), clear_rows=int(clear.sum()))
    # observed (r2): 7.5e-3-8.8e-3 rel; argmax on all 48 rows 0.94-1.0 from run to run — synthetic weights leave
    # near-ties among 151,936 logits, and the split-K GEMMs' atomic order varies per run — so the argmax is
    # required on the rows with a clear margin (top-2 gap > 2 % of the range), as for the decode logits
    assert e < 1.8e-2
    assert (got.argmax(1) == ref.argmax(1))[clear].all()


def test_real_forced_decode_logits(pair):
    """the oracle's greedy tokens fed back one per step through the decode path (GEMV rows, fused decode attention)"""
    arch, _, s, o = pair
    audio = clip(2.5, 13)
    ids, remb = _prompt_embeds(o, audio)
    kv = oracle.KV(o, 256)
    toks, ref = kv.generate(ids, SP["tok_audio_pad"], remb, eos=(), max_new=8, force_len=8, want_logits=True)
    got = s.forced_logits(audio, toks[:-1])
    assert got.shape == ref.shape
    e = rel_err(got, ref)
    clear = np.array([not _near_tie(r) for r in ref])
    record(f"real_forced_logits[{arch}]", logits_rel=e, clear_rows=int(clear.sum()))
    # observed (r2): 6.9e-3 / 7.3e-3 rel (0.6B / 1.7B), argmax equal on all 8 rows
    assert e < 1.5e-2
    assert (got.argmax(1) == ref.argmax(1))[clear].all()


def test_real_greedy_run_matches_oracle(pair):
    """Session.run (natural EOS) against the oracle's greedy decode of the same audio"""
    arch, _, s, o = pair
    audio = clip(3.0, 14)
    ids, remb = _prompt_embeds(o, audio)
    kv = oracle.KV(o, 256)
    ref, lg = kv.generate(ids, SP["tok_audio_pad"], remb, eos=(SP["tok_eos0"], SP["tok_eos1"]), max_new=12,
                          want_logits=True)
    res = s.run(audio, max_new_tokens=12)
    got = np.array(res.tokens, np.int32)
    assert res.n_audio_tokens == remb.shape[0]
    n = min(len(got), len(ref))
    div = next((i for i in range(n) if got[i] != ref[i]), n)
    record(f"real_greedy[{arch}]", first_divergence=div, n=n)
    if div < n:
        assert _near_tie(lg[div]), f"divergence at {div} without a near-tie"
    assert div >= min(8, n)


def test_real_greedy_long_matches_oracle(pair):
    """verdict r2 'what's weak' 2: greedy parity over a realistic transcript length — 64 tokens of an 8 s clip (the
    reference's ~8 tokens per audio second) against the oracle's greedy decode, every token equal up to the first
    near-tie of the oracle's own logits (synthetic weights do not emit EOS within a transcript's length, so the
    budget, not EOS, ends both runs; the EOS-ended budget logic is test_model_gpu.py's)"""
    arch, _, s, o = pair
    audio = clip(8.0, 23)
    ids, remb = _prompt_embeds(o, audio)
    kv = oracle.KV(o, 512)
    ref, lg = kv.generate(ids, SP["tok_audio_pad"], remb, eos=(SP["tok_eos0"], SP["tok_eos1"]), max_new=64,
                          want_logits=True)
    res = s.run(audio, max_new_tokens=64)
    got = np.array(res.tokens, np.int32)
    n = min(len(got), len(ref))
    div = next((i for i in range(n) if got[i] != ref[i]), n)
    record(f"real_greedy_long[{arch}]", first_divergence=div, n=n)
    # observed on MI355X (r3, build f5148bb7): all 64 tokens equal at both sizes (profiles/r3z_greedy_long.jsonl)
    if div < n:
        assert _near_tie(lg[div]), f"divergence at {div} without a near-tie"
    assert div >= min(32, n)
    assert n == 64 or len(got) == len(ref)


def test_real_decode_fusion_bit_identical(pair, monkeypatch):
    """the 1–4-row decode with the norms / SwiGLU in the GEMV prologues (default) against the separate launches
    (QASR_NO_DEC_FUSE=1): teacher-forced logits equal bit for bit, and 40 forced decode steps give the same tokens
    (verdict r1 item 5: tokens identical to the previous build)"""
    from qasr import _lib

    arch, m, s, _ = pair
    monkeypatch.setenv("QASR_NO_DEC_FUSE", "1")
    s2 = m.session(kv_type="f16", n_ctx=4096)
    monkeypatch.delenv("QASR_NO_DEC_FUSE")
    # the prefill / encoder GEMMs split K with float atomics (run-to-run last-ulp noise): compare without
    _lib.check(_lib.load().qasr_set_deterministic(1))
    try:
        audio = clip(5.0, 16)
        forced = np.array([900 + 41 * i for i in range(5)], np.int32)
        assert np.array_equal(s.forced_logits(audio, forced), s2.forced_logits(audio, forced))
        a = s.run(audio, force_tokens_per_s=8).tokens
        b = s2.run(audio, force_tokens_per_s=8).tokens
        assert len(a) == 41 and a == b
    finally:
        _lib.check(_lib.load().qasr_set_deterministic(1))   # the default
        s2.close()


def test_real_deterministic_mode_repeats(pair):
    """deterministic mode: two runs of the same request give bit-identical logits"""
    from qasr import _lib

    arch, _, s, _ = pair
    audio = clip(2.0, 17)
    forced = np.array([700, 701], np.int32)
    _lib.check(_lib.load().qasr_set_deterministic(1))
    try:
        assert np.array_equal(s.forced_logits(audio, forced), s.forced_logits(audio, forced))
    finally:
        _lib.check(_lib.load().qasr_set_deterministic(1))   # the default


def test_real_batch_equals_single_and_oracle(pair):
    """1.7B: 8 segments of 1-4.5 s decoded together (rows > 4: MFMA decode GEMMs, step graphs, shrinking batch) give
    the tokens of the 8 single runs (GEMV path); segment 0 also against the oracle.  A divergence is allowed only at
    a near-tie of the oracle's logits."""
    arch, _, s, o = pair
    if arch != "qwen3-asr-1.7b":
        pytest.skip("batched decode at the C4 model only")
    clips = [clip(1.0 + 0.5 * i, 20 + i) for i in range(8)]
    batch = [r.tokens for r in s.run_batch(clips, max_new_tokens=10)]
    singles = [s.run(c, max_new_tokens=10).tokens for c in clips]
    diffs = [i for i in range(8) if batch[i] != singles[i]]
    for i in diffs:   # must be a near-tie: check against the oracle's logits at the first divergence
        ids, remb = _prompt_embeds(o, clips[i])
        ref, lg = oracle.KV(o, 256).generate(ids, SP["tok_audio_pad"], remb, eos=(SP["tok_eos0"], SP["tok_eos1"]),
                                             max_new=10, want_logits=True)
        a, b = batch[i], singles[i]
        d = next(j for j in range(min(len(a), len(b)) + 1) if j >= min(len(a), len(b)) or a[j] != b[j])
        assert d < len(lg) and _near_tie(lg[d]), f"segment {i}: batch/single diverge at {d} without a near-tie"
    ids, remb = _prompt_embeds(o, clips[0])
    ref, lg = oracle.KV(o, 256).generate(ids, SP["tok_audio_pad"], remb, eos=(SP["tok_eos0"], SP["tok_eos1"]),
                                         max_new=10, want_logits=True)
    n = min(len(batch[0]), len(ref))
    div = next((j for j in range(n) if batch[0][j] != ref[j]), n)
    record(f"real_batch[{arch}]", batch_vs_single_mismatches=len(diffs), seg0_first_divergence=div, n=n)
    if div < n:
        assert _near_tie(lg[div])
    assert div >= min(6, n)


def test_real_batch_c4_scale(pair):
    """C4 at scale (1.7B, 64 segments of U[2,12] s like bench.py, 8 forced tokens per audio-second: up to 97 tokens,
    EOS ignored): the batch's token streams against the 64 single runs, and 8 segments (the two shortest, the longest,
    five length quantiles) against the oracle.  The mismatch count and every first divergence are recorded ($QASR_PARITY_LOG); a divergence is allowed
    only at a near-tie (0.5 % of the row's range) of the single run's teacher-forced logits (batch vs single) or of
    the oracle's logits (batch vs oracle)."""
    arch, _, s, o = pair
    if arch != "qwen3-asr-1.7b":
        pytest.skip("C4 is quoted on the 1.7B model")
    rng = np.random.default_rng(11)
    secs = rng.uniform(2.0, 12.0, size=64)
    clips = [clip(float(x), 500 + i) for i, x in enumerate(secs)]
    batch = [r.tokens for r in s.run_batch(clips, force_tokens_per_s=8)]
    singles = [s.run(c, force_tokens_per_s=8).tokens for c in clips]
    for i, c in enumerate(clips):
        n_want = int(round(8 * c.size / 16000.0)) + 1
        assert len(batch[i]) == n_want and len(singles[i]) == n_want, (i, len(batch[i]), len(singles[i]), n_want)
    # every prefill runs the row-count-independent order and the first token's projection the 1-row arithmetic
    # (engine.cpp run_batch): the first tokens are the single runs' exactly, with no near-tie allowance
    assert [b[0] for b in batch] == [x[0] for x in singles]
    divs = {}
    for i in range(64):
        a, b = batch[i], singles[i]
        d = next((j for j in range(len(a)) if a[j] != b[j]), None)
        if d is None:
            continue
        divs[i] = d
        lg = s.forced_logits(clips[i], np.asarray(b[:d], np.int32))   # row d: the single path's logits at the split
        assert _near_tie(lg[d]), f"segment {i}: batch/single diverge at token {d} of {len(a)} without a near-tie"
    # the oracle on 8 segments (forced length, EOS ignored, as the batch): the two shortest, the longest (12 s class:
    # ~97 tokens, key ranges past the 256-key split) and five at evenly spaced length quantiles between them
    order = np.argsort(secs)
    pick = [int(i) for i in order[:2]] + [int(order[-1])] + [int(order[q]) for q in (13, 25, 38, 50, 57)]
    oracle_divs = []
    for i in pick:
        ids, remb = _prompt_embeds(o, clips[i])
        n_new = len(batch[i])
        ref, lg = oracle.KV(o, len(ids) + n_new + 8).generate(ids, SP["tok_audio_pad"], remb, eos=(), max_new=n_new,
                                                              force_len=n_new, want_logits=True)
        d = next((j for j in range(n_new) if batch[i][j] != ref[j]), n_new)
        oracle_divs.append((int(i), d, n_new))
        if d < n_new:
            assert _near_tie(lg[d]), f"segment {i}: batch/oracle diverge at token {d} without a near-tie"
        assert d >= min(8, n_new), (i, d)
    record(f"real_batch_c4[{arch}]", segments=64, tokens=int(sum(len(b) for b in batch)),
           batch_vs_single_mismatched_segments=len(divs), first_divergences=sorted(divs.items()),
           oracle_first_divergence=oracle_divs,
           oracle_mismatched_segments=sum(1 for _, d, n in oracle_divs if d < n),
           oracle_tokens_compared=int(sum(n for *_, n in oracle_divs)))


def test_real_batch_c4_full(pair):
    """C4 exactly as bench.py runs it (1.7B, its 256 U[2,12] s segments, seed 1, 8 forced tokens per audio-second):
    the 256-segment batch's token streams against the 256 single runs (session.run, qwen3_asr_server.py:321) — first
    tokens equal with no allowance (stable-order prefill), a later divergence only at a near-tie of the single path's
    teacher-forced logits.  Observed on MI355X: 0 of 256 segments diverge, 14,577 tokens
    (profiles/r5_parity_c4_full_256.json, tools/diag_c4full.py)."""
    from bench import make_workload

    arch, _, s, _ = pair
    if arch != "qwen3-asr-1.7b":
        pytest.skip("C4 is quoted on the 1.7B model")
    clips = make_workload(1, 0, seed=1, total=256)
    batch = [r.tokens for r in s.run_batch(clips, force_tokens_per_s=8)]
    singles = [s.run(c, force_tokens_per_s=8).tokens for c in clips]
    assert [b[0] for b in batch] == [x[0] for x in singles]
    divs = {}
    for i in range(len(clips)):
        d = next((j for j in range(len(batch[i])) if batch[i][j] != singles[i][j]), None)
        if d is None:
            continue
        divs[i] = d
        lg = s.forced_logits(clips[i], np.asarray(singles[i][:d], np.int32))
        assert _near_tie(lg[d]), f"segment {i}: batch/single diverge at token {d} without a near-tie"
    record(f"real_batch_c4_full[{arch}]", segments=len(clips), tokens=int(sum(len(b) for b in batch)),
           batch_vs_single_mismatched_segments=len(divs), first_divergences=sorted(divs.items()))


def test_real_batch_invariant(pair):
    """batch invariance (Session.set_batch_invariant): 1.7B, 48 segments of U[2,12] s (more than 32 decode
    rows: two exact-row chunks per linear; the longest key ranges pass 256 keys: the split attention), 8 forced tokens
    per audio-second — every segment's token stream equals its default single run's (session.run,
    qwen3_asr_server.py:321) EXACTLY, with no near-tie allowance, and a batch of other composition (the odd segments
    alone) gives the same streams again"""
    arch, _, s, _ = pair
    if arch != "qwen3-asr-1.7b":
        pytest.skip("C4 is quoted on the 1.7B model")
    rng = np.random.default_rng(13)
    secs = rng.uniform(2.0, 12.0, size=48)
    secs[5] = 12.0   # 15 prompt + 156 audio + 97 generated tokens: key ranges past the 256-key split threshold
    clips = [clip(float(x), 900 + i) for i, x in enumerate(secs)]
    singles = [s.run(c, force_tokens_per_s=8).tokens for c in clips]   # the default single-utterance path
    s.set_batch_invariant(True)
    try:
        batch = [r.tokens for r in s.run_batch(clips, force_tokens_per_s=8)]
        odd = [r.tokens for r in s.run_batch(clips[1::2], force_tokens_per_s=8)]
    finally:
        s.set_batch_invariant(False)
    for i, c in enumerate(clips):
        assert len(batch[i]) == len(singles[i]) == int(round(8 * c.size / 16000.0)) + 1, i
    mism = [i for i in range(48) if batch[i] != singles[i]]
    mism_odd = [i for i in range(1, 48, 2) if odd[i // 2] != singles[i]]
    record(f"real_batch_invariant[{arch}]", segments=48, tokens=int(sum(len(b) for b in batch)),
           batch_vs_single_mismatched_segments=len(mism), odd_batch_mismatched_segments=len(mism_odd))
    assert not mism and not mism_odd, (mism, mism_odd)


def test_real_mxfp8_against_q8(pair):
    """1.7B MXFP8 precision mode (C5; tolerance parity only) against the Q8 path on teacher-forced logits"""
    from qasr.transcribe_cpp import Model

    arch, _, s, o = pair
    if arch != "qwen3-asr-1.7b":
        pytest.skip("C5 precision is quoted on the 1.7B model")
    audio = clip(2.5, 15)
    forced = np.array([1000 + 37 * i for i in range(6)], np.int32)
    ref = s.forced_logits(audio, forced)
    mx = Model.synthetic(arch, seed=SEED)
    try:
        mx.set_precision("mxfp8")
        ms = mx.session(kv_type="f16", n_ctx=1024)
        got = ms.forced_logits(audio, forced)
        ms.close()
    finally:
        mx.close()
    span = np.abs(ref).max()
    e = float(np.abs(got - ref).max() / span)
    top2 = np.sort(ref, 1)[:, -2:]
    clear = (top2[:, 1] - top2[:, 0]) > 0.1 * span
    agree = float((got.argmax(1) == ref.argmax(1)).mean())
    record(f"real_mxfp8[{arch}]", logits_rel_vs_q8=e, argmax_agree=agree, clear_rows=int(clear.sum()))
    # observed: 3.95e-2 of the logit range (r2), 8.8e-2 with r3's peaked synthetic vocabulary (row gains up to ~7×:
    # the largest logits carry the largest e4m3 rounding); argmax equal on all 7 rows
    assert e < 1.5e-1
    assert (got.argmax(1) == ref.argmax(1))[clear].all()


def test_real_draft_verify_pass_bit_identical(pair):
    """exact-row contract at the real shapes: a forced continuation of 1–32 tokens fed as ONE draft
    verify pass gives the same logits, bit for bit, as one decode step per token — including a 20 s prompt, whose
    > 256 keys split each row's key range over workgroups exactly as a single row's"""
    arch, _, s, _ = pair
    for secs, seed, ns in ((4.0, 31, (2, 9, 32)), (20.0, 32, (1, 17))):
        audio = clip(secs, seed)
        for n in ns:
            forced = np.array([1000 + 37 * i for i in range(n)], np.int32)
            assert np.array_equal(s.forced_logits(audio, forced), s.forced_logits(audio, forced, one_pass=True)), \
                (secs, n)


def _interim_windows(seconds=17.0, seed=40):
    """the app's interim loop (interim.rs:135-156): the window grows from the utterance start while it is shorter than
    12 s, then slides (the last 12 s); ticks every 1.4 s here, plus the final request over the whole recording"""
    rec = np.concatenate([clip(5.0, seed), clip(4.0, seed + 1), clip(8.0, seed + 2)])[: int(seconds * 16000)]
    out, t = [], 1.4
    while t < seconds:
        n = int(t * 16000)
        out.append(rec[max(0, n - 12 * 16000): n])
        t += 1.4
    return out + [rec, rec]


def test_real_streaming_bit_identical(pair):
    """the product transcript is a pure function of (weights, audio).  An interim replay across the
    12 s boundary (growing, then sliding windows, then the final request, repeated) through a session with prompt-
    lookup drafts and the encoder cache on gives the SAME audio-embedding rows and tokens as a plain session, for
    draft noise 0 / 20 / 50 % (acceptance below the degenerate 100 % of synthetic transcripts), and the plain
    session repeats itself bit for bit."""
    arch, m, s, _ = pair
    windows = _interim_windows()
    H = m.hparams["txt_h"]
    plain = [s.run(w, max_new_tokens=40) for w in windows]
    plain_emb = [None] * len(windows)
    for i, w in enumerate(windows[-3:]):   # the plain session repeats itself (deterministic by default)
        r = s.run(w, max_new_tokens=40)
        assert r.tokens == plain[len(windows) - 3 + i].tokens
    for noise in (0.0, 0.2, 0.5):
        st = m.session(kv_type="f16", n_ctx=4096)
        st.set_draft(True)
        st.set_encoder_cache(True)
        st.set_draft_noise(noise, seed=5)
        for i, w in enumerate(windows):
            got = st.run(w, max_new_tokens=40)
            assert got.tokens == plain[i].tokens, (noise, i)
            if noise == 0.0:
                if plain_emb[i] is None:
                    s.run(w, max_new_tokens=1)
                    plain_emb[i] = s.audio_embeds().reshape(-1, H)
                assert np.array_equal(st.audio_embeds().reshape(-1, H), plain_emb[i]), i
        ds, ec = st.draft_stats(), st.encoder_cache_stats()
        record(f"real_streaming[{arch}]", noise=noise, **{f"draft_{k}": v for k, v in ds.items()},
               **{f"cache_{k}": v for k, v in ec.items()})
        assert ds["accepted"] > 0 and ec["windows_reused"] > 0, (ds, ec)
        if noise > 0:
            assert ds["proposed"] > ds["accepted"], ds
        st.close()


def test_real_teacher_forced_100_tokens(pair):
    """100 teacher-forced decode steps at 1.7B against the oracle — the oracle's own greedy tokens fed
    back one per step through the GPU decode path (GEMV rows, fused split attention past 256 keys): every row within
    the logit bound, the argmax equal on every row with a clear margin (top-2 gap > 0.5 % of the row's range), and
    the clear rows ≥ 80 % of all (the fraction is recorded)."""
    arch, _, s, o = pair
    if arch != "qwen3-asr-1.7b":
        pytest.skip("C3/C4 model")
    audio = clip(6.0, 41)
    ids, remb = _prompt_embeds(o, audio)
    kv = oracle.KV(o, len(ids) + 128)
    toks, ref = kv.generate(ids, SP["tok_audio_pad"], remb, eos=(), max_new=100, force_len=100, want_logits=True)
    got = s.forced_logits(audio, toks[:-1])
    assert got.shape == ref.shape == (100, o.cfg["vocab"])
    e = rel_err(got, ref)
    clear = np.array([not _near_tie(r) for r in ref])
    agree = got.argmax(1) == ref.argmax(1)
    record(f"real_forced_100[{arch}]", logits_rel=e, clear_frac=float(clear.mean()), argmax_agree=float(agree.mean()),
           argmax_agree_clear=float(agree[clear].mean()))
    assert e < 2e-2
    assert agree[clear].all(), np.nonzero(~agree & clear)
    assert clear.mean() >= 0.8


def test_real_fused_norm_and_xr_bit_identical(pair, monkeypatch):
    """round 5's ≤ 32-row decode launches — the exact-row linears as per-phase xr launches and the RMSNorm fused into
    the residual launches' tails (opt-in QASR_XR_NORM=1) — against the round-4 launch chain (QASR_NO_XR=1:
    gemm_exact_rows + rmsnorm_q8): a batch-invariant batch of 20 segments (rows 20 → 1) gives the same token streams, and the same
    streams as the segments' single runs"""
    arch, m, s, _ = pair
    rng = np.random.default_rng(31)
    secs = rng.uniform(2.0, 8.0, size=20)
    clips = [clip(float(x), 700 + i) for i, x in enumerate(secs)]
    singles = [s.run(c, force_tokens_per_s=8).tokens for c in clips[:6]]
    s.set_batch_invariant(True)
    try:
        monkeypatch.setenv("QASR_XR_NORM", "1")
        new = [r.tokens for r in s.run_batch(clips, force_tokens_per_s=8)]
        monkeypatch.delenv("QASR_XR_NORM")
        monkeypatch.setenv("QASR_NO_XR", "1")
        s2 = m.session(kv_type="f16", n_ctx=4096)
        s2.set_batch_invariant(True)
        old = [r.tokens for r in s2.run_batch(clips, force_tokens_per_s=8)]
        s2.close()
    finally:
        s.set_batch_invariant(False)
    assert new == old
    assert new[:6] == singles


def test_real_c5_mxfp8_longform_against_q8(pair):
    """C5 (BASELINE configs[4]: 1.7B with MXFP8 MFMA weights, long-form) at its shape: a 300 s recording (seed 2, the
    C5 generator) through the long-form pipeline (qasr.longform: FireRedVAD probabilities, the reference's segmenter,
    one batch of every speech segment), in MXFP8 precision against the Q8 path.  The batch's decode steps run 5–64
    rows, so the block-scaled MFMA GEMMs of the BATCHED decode are exercised (1–4-row steps keep the Q8 GEMVs).
      * VAD probabilities and segments bit-identical between the two runs (precision does not touch the VAD);
      * every segment's first token (the prompt's argmax, batched prefill) equal wherever the Q8 row is clear, and
        its prompt logits within the MXFP8 tolerance;
      * teacher-forced logits through the batched decode (qasr_session_forced_logits_batch: every segment fed the Q8
        batch's own token stream) at 3 segments — the longest, the median, the shortest — within the tolerance, argmax
        equal on clear rows;
      * the free-running token streams' mismatch count recorded (MXFP8 is tolerance parity: the reference has no fp8
        path).
    Tolerance: TOL = 0.35 of the row's max |logit| — e4m3 element rounding of every weight and activation over 28
    layers of the synthetic (untrained) model; observed on MI355X (r6): 0.227 on the prompt rows of these segments
    (2.5–8 s of speech, 100–200 prompt rows: the 2.5 s clip of test_real_mxfp8_against_q8 sees 8.8e-2); a row is
    clear when its Q8 top-2 gap exceeds 2·TOL of that span (no error within the tolerance can flip it).  The free-
    running first-token and stream agreement is recorded, not bounded: MXFP8 is tolerance parity only."""
    TOL = 0.35
    from bench import recording
    from qasr import longform
    from qasr.firered_vad import FireRedVad
    from qasr.transcribe_cpp import Model

    arch, _, s, _ = pair
    if arch != "qwen3-asr-1.7b":
        pytest.skip("C5 is quoted on the 1.7B model")
    rec = recording(300.0, seed=2)
    vad = FireRedVad()

    def pipeline_segments():
        p = longform.shard_probabilities(vad, rec, 0, 1)
        return p, longform.segments(p, rec.size)

    p_q8, segs = pipeline_segments()
    mx = Model.synthetic(arch, seed=SEED)
    try:
        mx.set_precision("mxfp8")
        ms = mx.session(kv_type="f16", n_ctx=4096)
        p_mx, segs_mx = pipeline_segments()
        assert np.array_equal(p_q8.view(np.uint32), p_mx.view(np.uint32)) and segs == segs_mx
        n = len(segs)
        assert n >= 20, n
        clips = [rec[a:b] for a, b in segs]
        q8_tok = [r.tokens for r in s.run_batch(clips, force_tokens_per_s=8)]
        mx_tok = [r.tokens for r in ms.run_batch(clips, force_tokens_per_s=8)]
        # prompt logits of every segment (batched prefill), first tokens
        allw = np.arange(n, dtype=np.int32)
        empty = np.zeros((n, 0), np.int32)
        pq = s.forced_logits_batch(clips, empty, allw)[:, 0]
        pm = ms.forced_logits_batch(clips, empty, allw)[:, 0]

        def row_err(got, ref):
            return np.abs(got - ref).max(1) / np.abs(ref).max(1)

        def clear_rows(ref, frac=2 * TOL):
            # a row whose argmax no error within the tolerance can flip: top-2 gap above twice the per-logit bound
            top2 = np.sort(ref, 1)[:, -2:]
            return (top2[:, 1] - top2[:, 0]) > frac * np.abs(ref).max(1)

        e_prompt = float(row_err(pm, pq).max())
        cq = clear_rows(pq)
        near = clear_rows(pq, 0.005 * 2)   # rows whose Q8 argmax is not a near-tie of the Q8 batch's own order
        first_mism = [i for i in range(n) if mx_tok[i][0] != q8_tok[i][0]]
        record(f"real_c5_mxfp8_longform_prompt[{arch}]", segments=n, prompt_logits_rel=e_prompt,
               first_token_mismatches=len(first_mism), clear_rows=int(cq.sum()),
               first_token_mismatches_clear=len([i for i in first_mism if cq[i]]))
        # the tf hook's prompt rows == the batch run's first tokens (same batch, same order; near-ties aside)
        assert all(q8_tok[i][0] == int(pq[i].argmax()) for i in range(n) if near[i])
        assert all(mx_tok[i][0] == int(pm[i].argmax()) for i in range(n) if clear_rows(pm, 0.01)[i])
        assert e_prompt < TOL, e_prompt
        assert not [i for i in first_mism if cq[i]], first_mism
        # teacher-forced decode logits through the batched steps
        lens = np.array([len(t) for t in q8_tok])
        order = np.argsort(lens, kind="stable")
        want = np.array([order[-1], order[n // 2], order[0]], np.int32)
        nf = int(lens.max()) - 1
        forced = np.array([(t + [t[-1]] * nf)[:nf] for t in q8_tok], np.int32)
        fq = s.forced_logits_batch(clips, forced, want)
        fm = ms.forced_logits_batch(clips, forced, want)
        errs, clear_n, argmax_bad = [], 0, 0
        for k, u in enumerate(want):
            rows = len(q8_tok[u])   # the rows past the segment's own stream are padding
            rq, rm = fq[k, :rows], fm[k, :rows]
            errs.append(float(row_err(rm, rq).max()))
            c = clear_rows(rq)
            clear_n += int(c.sum())
            argmax_bad += int((rm.argmax(1) != rq.argmax(1))[c].sum())
            # the hook feeds the Q8 batch's stream: its argmax reproduces that stream (the tf batch steps run other
            # row buckets than the free run, so near-ties of the GEMM order aside)
            nt = clear_rows(rq, 0.01)
            assert all(int(rq[j].argmax()) == q8_tok[u][j] for j in range(rows) if nt[j]), int(u)
        stream_mism = sum(1 for i in range(n) if mx_tok[i] != q8_tok[i])
        record(f"real_c5_mxfp8_longform[{arch}]", recording_s=300.0, segments=n,
               speech_s=round(sum(b - a for a, b in segs) / 16000.0, 1), max_rows=n,
               prompt_logits_rel=e_prompt, first_token_mismatches=len(first_mism),
               first_token_clear_rows=int(cq.sum()), tf_segments=[int(u) for u in want],
               tf_logits_rel=errs, tf_clear_rows=clear_n, tf_argmax_mismatch_clear=argmax_bad,
               stream_mismatched_segments=stream_mism, tokens=int(lens.sum()))
        assert max(errs) < TOL, errs
        assert argmax_bad == 0, argmax_bad
        ms.close()
    finally:
        mx.close()


_DUMP_CHILD = r"""
import json, os, sys
import numpy as np
sys.path.insert(0, os.path.join(sys.argv[1], "light-whisper_amd"))
sys.path.insert(0, sys.argv[1])
from qasr.transcribe_cpp import Model
from bench import speech_like
secs = json.loads(sys.argv[3])
clips = [speech_like(np.random.default_rng(600 + i), int(x * 16000)) for i, x in enumerate(secs)]
m = Model.synthetic(sys.argv[2], seed=7)
s = m.session(kv_type="f16", n_ctx=4096)
single = s.run(clips[0], force_tokens_per_s=8).tokens
s.set_batch_invariant(True)
batch = [r.tokens for r in s.run_batch(clips, force_tokens_per_s=8)]
s.close()
m.close()
print(json.dumps({"single": list(single), "batch": [list(b) for b in batch]}))
"""


def test_real_dump_mode_same_tokens(pair, tmp_path):
    """diagnosis dump mode (QASR_DUMP_DIR: every ≤ 32-row decode stage's rows written to files, the fused norms split
    off) computes the same tokens as a normal run — ADVICE r5: the exact-row path once skipped the down projection
    under dump.  The dump switch is read once per process, so the dumping run is a child process (eager passes,
    QASR_NO_GRAPH, as the diagnosis tools run); batch-invariant rows take the exact-row (xm) path"""
    import json
    import os
    import subprocess
    import sys

    arch, _, s, _ = pair
    if arch != "qwen3-asr-0.6b":
        pytest.skip("one architecture is enough for the dump switch")
    secs = [2.0, 2.6, 3.1]
    clips = [clip(x, 600 + i) for i, x in enumerate(secs)]
    single = list(s.run(clips[0], force_tokens_per_s=8).tokens)
    s.set_batch_invariant(True)
    try:
        batch = [list(r.tokens) for r in s.run_batch(clips, force_tokens_per_s=8)]
    finally:
        s.set_batch_invariant(False)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, QASR_DUMP_DIR=str(tmp_path), QASR_NO_GRAPH="1")
    out = subprocess.run([sys.executable, "-c", _DUMP_CHILD, root, arch, json.dumps(secs)], env=env,
                         capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    got = json.loads(out.stdout.strip().splitlines()[-1])
    dumps = len(os.listdir(tmp_path))
    record(f"real_dump_mode[{arch}]", dump_files=dumps)
    assert dumps > 0
    assert got["single"] == single
    assert got["batch"] == batch
