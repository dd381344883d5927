// `engine longform`: the C5 long-form pipeline with no PyTorch anywhere — the host path a
// Rust process drives over the C ABI, in C++ here because the image has no Rust toolchain.  One
// process per GPU (RANK / WORLD_SIZE / LOCAL_RANK as torchrun sets them):
//   1. the 128-byte RCCL unique id handed over through a file (qasr/dist.py file_exchange's protocol:
//      <QASR_RDV_DIR|TMPDIR|/tmp>/qasr_uid_<TORCHELASTIC_RUN_ID>_<MASTER_PORT>_<launcher pid>.bin (or
//      qasr_uid_<QASR_RDV_KEY>.bin), written under a temporary name and
//      renamed), qasr_dist_init;
//   2. rank 0 loads (or generates) the model, every other rank opens a shell of the same layout and receives the
//      weight blob in ONE broadcast (qasr_dist_broadcast_weights: checksums compared);
//   3. FireRedVAD on this rank's contiguous frame range plus a ±160-frame halo — the DFSMN's receptive field, so its
//      core probabilities are the bits of one pass over the whole recording (qasr/longform.py) — and an all-gather of
//      the probabilities (qasr_dist_gather_tokens on their bit patterns);
//   4. the reference's post-processing on the full vector, identically on every rank
//      (qasr_vad_timestamps_from_probabilities = firered_vad.py:121-191), the segments LPT-assigned by length;
//   5. this rank's segments (time order) through ONE qasr_run_batch;
//   6. the token streams all-gathered (qasr_dist_gather_tokens); rank 0 detokenises, splits language / text
//      (qasr_parse_transcript) and prints one JSON object.
// The reference handles one short utterance per request and has no long-form or multi-GPU mode.
// Failure agreement: once the communicator exists, every step that precedes a collective (model load, VAD, the ASR
// batch) is a stage whose local outcome all ranks agree on first (qasr_dist_agree: one int32 all-gather) — a rank
// whose stage failed makes EVERY rank exit non-zero with the failing rank's reason instead of leaving the others
// blocked in the collective (the reference sees one crashed process, funasr_service.rs:1367-1385).  The stages can be
// failed on purpose for tests: QASR_FAIL_STAGE=model|vad|asr [QASR_FAIL_RANK=r, default every rank].  At world 1,
// QASR_LONGFORM_COMM=1 opens a one-rank communicator so the same agreement path runs.  A rank that never joins the
// communicator (QASR_FAIL_STAGE=init injects it: the rank exits before qasr_dist_init) or dies inside a collective
// makes the others fail at the communicator's deadline (qasr_dist_init_deadline, QASR_DIST_TIMEOUT_MS) instead of
// hanging; a failure before the communicator exists goes through the unique-id hand-off (rank 0 leaves a ".fail"
// marker, so the other ranks stop polling at once; rank 0 clears a stale marker before it publishes).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <numeric>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../../include/qasr.h"
#include "json.h"

namespace {

using qjson::Value;

struct Fail : std::runtime_error {
    using std::runtime_error::runtime_error;
};

void ck(int rc, const char* what) {
    if (rc != QASR_OK) throw Fail(std::string(what) + ": " + qasr_last_error());
}

int env_int(const char* name, int def) {
    const char* e = getenv(name);
    return e && *e ? atoi(e) : def;
}

double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// qasr/dist.py file_exchange: rank 0 publishes, the others poll (same path, so a Python rank and a native rank can
// share one launch)
std::string uid_path() {
    const char* dir = getenv("QASR_RDV_DIR");
    if (!dir || !*dir) dir = getenv("TMPDIR");
    if (!dir || !*dir) dir = "/tmp";
    if (const char* k = getenv("QASR_RDV_KEY"); k && *k) return std::string(dir) + "/qasr_uid_" + k + ".bin";
    const char* run = getenv("TORCHELASTIC_RUN_ID");
    const char* port = getenv("MASTER_PORT");
    // + the launcher's pid (torchrun's agent is every rank's parent): never a stale file of an earlier launch
    return std::string(dir) + "/qasr_uid_" + (run && *run ? run : "run") + "_" + (port && *port ? port : "0") + "_" +
           std::to_string(getppid()) + ".bin";
}

// RCCL prints its version banner on stdout when it first initialises; stdout is this command's JSON channel, so the
// RCCL calls run with fd 1 pointed at stderr (in the executable, not in the library: qasr.h "Multi-GPU")
struct StdoutToStderr {
    int saved = -1;
    StdoutToStderr() {
        fflush(stdout);
        saved = dup(1);
        if (saved >= 0) dup2(2, 1);
    }
    ~StdoutToStderr() {
        fflush(stdout);
        if (saved >= 0) dup2(saved, 1), close(saved);
    }
};

// rank 0 could not create or publish the id: a marker next to the id file, so the other ranks stop polling at once
void publish_uid_failure(const std::string& path) {
    if (FILE* f = fopen((path + ".fail").c_str(), "wb")) fclose(f);
}

void exchange_uid(uint8_t id[128], int rank, const std::string& path, double timeout_s) {
    if (rank == 0) {
        remove((path + ".fail").c_str());   // a stale marker of an earlier launch with the same key
        const std::string tmp = path + "." + std::to_string(getpid()) + ".tmp";
        FILE* f = fopen(tmp.c_str(), "wb");
        if (!f || fwrite(id, 1, 128, f) != 128) throw Fail("unique id: cannot write " + tmp);
        fflush(f);
        fsync(fileno(f));
        fclose(f);
        if (rename(tmp.c_str(), path.c_str()) != 0) throw Fail("unique id: cannot rename to " + path);
        return;
    }
    const double t0 = now_ms();
    for (;;) {
        if (FILE* f = fopen(path.c_str(), "rb")) {
            const size_t got = fread(id, 1, 128, f);
            fclose(f);
            if (got == 128) return;
        }
        if (FILE* f = fopen((path + ".fail").c_str(), "rb")) {
            fclose(f);
            throw Fail("rank " + std::to_string(rank) + ": rank 0 failed to publish the unique id");
        }
        if (now_ms() - t0 > timeout_s * 1e3) throw Fail("rank " + std::to_string(rank) + ": no unique id at " + path);
        std::this_thread::sleep_for(std::chrono::milliseconds(10));
    }
}

// Kaldi snip_edges frames (firered_vad.py:87-104: 25 ms windows, 10 ms shift at 16 kHz) and the halo shard
constexpr int64_t kShift = 160, kLen = 400, kHalo = 160;
int64_t n_frames(int64_t n) { return n < kLen ? 0 : 1 + (n - kLen) / kShift; }

// longest-processing-time assignment (bench.py lpt_shard): stable order by decreasing length, each to the least loaded
std::vector<std::vector<int>> lpt_shard(const std::vector<int64_t>& len, int world) {
    std::vector<int> order(len.size());
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return len[a] > len[b]; });
    std::vector<double> load(world, 0.0);
    std::vector<std::vector<int>> out(world);
    for (int i : order) {
        const int r = (int)(std::min_element(load.begin(), load.end()) - load.begin());
        out[r].push_back(i);
        load[r] += (double)len[i];
    }
    for (auto& v : out) std::sort(v.begin(), v.end());   // time order within a rank
    return out;
}

// every rank's int32 array to every rank, in rank order (two-phase: sizes, then payload)
std::vector<int32_t> all_gather_i32(qasr_comm* c, const std::vector<int32_t>& mine, int world,
                                    std::vector<int32_t>& per_rank) {
    const int32_t n = (int32_t)mine.size();
    std::vector<int32_t> rank_segs(world);
    size_t ns = 0, nt = 0;
    ck(qasr_dist_gather_tokens(c, &n, 1, mine.data(), rank_segs.data(), nullptr, 0, nullptr, 0, &ns, &nt),
       "gather (sizes)");
    std::vector<int32_t> lens(ns), flat(std::max<size_t>(nt, 1));
    ck(qasr_dist_gather_tokens(c, &n, 1, mine.data(), rank_segs.data(), lens.data(), lens.size(), flat.data(),
                               flat.size(), &ns, &nt),
       "gather");
    per_rank.assign(lens.begin(), lens.end());   // one array per rank
    flat.resize(nt);
    return flat;
}

}  // namespace

// argv: the arguments after "longform"; engine: the model id; gguf: resolved GGUF path ("" = synthetic weights)
int longform_main(const std::string& engine, const std::string& gguf, int argc, char** argv) {
    int force_tps = 0, max_new = 0;
    bool inv = false;
    std::string wav;
    for (int i = 0; i < argc; i++) {
        const std::string a = argv[i];
        if (a == "--force-tps" && i + 1 < argc) force_tps = atoi(argv[++i]);
        else if (a == "--max-new" && i + 1 < argc) max_new = atoi(argv[++i]);
        else if (a == "--batch-invariant") inv = true;
        else if (a == "--engine" && i + 1 < argc) i++;
        else if (!a.empty() && a[0] != '-') wav = a;
        else {
            fprintf(stderr, "engine longform: unknown argument %s\n", a.c_str());
            return 2;
        }
    }
    if (wav.empty()) {
        fprintf(stderr, "usage: engine longform --engine <id> [--force-tps K] [--max-new N] [--batch-invariant] "
                        "recording.wav  (RANK / WORLD_SIZE / LOCAL_RANK for N GPUs)\n");
        return 2;
    }
    const int rank = env_int("RANK", 0), world = env_int("WORLD_SIZE", 1), local = env_int("LOCAL_RANK", rank);
    qasr_comm* comm = nullptr;
    qasr_model* model = nullptr;
    qasr_session* sess = nullptr;
    qasr_vad* vad = nullptr;
    std::vector<qasr_result> res;
    int rc = 0;
    try {
        if (world < 1 || rank < 0 || rank >= world) throw Fail("bad RANK / WORLD_SIZE");
        ck(qasr_set_device(local), "device");
        const double t_start = now_ms();
        Value info = Value::object();
        if (world > 1 || env_int("QASR_LONGFORM_COMM", 0) != 0) {
            uint8_t id[128] = {0};
            const std::string path = uid_path();
            if (rank == 0) {
                try {
                    {
                        StdoutToStderr quiet;
                        ck(qasr_dist_unique_id(id, sizeof id), "unique id");
                    }
                    exchange_uid(id, rank, path, 600.0);
                } catch (...) {
                    publish_uid_failure(path);
                    throw;
                }
            } else {
                exchange_uid(id, rank, path, 600.0);
            }
            const char* inj = getenv("QASR_FAIL_STAGE");
            const int inj_rank = env_int("QASR_FAIL_RANK", -1);
            if (inj && strcmp(inj, "init") == 0 && (inj_rank < 0 || inj_rank == rank))
                throw Fail("injected failure (QASR_FAIL_STAGE=init): this rank never joins the communicator");
            {
                StdoutToStderr quiet;   // RCCL's version banner must not reach the JSON channel
                const int irc = qasr_dist_init(id, rank, world, local, &comm);
                if (irc != QASR_OK) {
                    // a rank that never joined (deadline, QASR_DIST_TIMEOUT_MS): the init thread is abandoned inside
                    // RCCL, so leave without runtime teardown (include/qasr.h qasr_dist_init_deadline)
                    fprintf(stderr, "engine longform (rank %d): communicator: %s\n", rank, qasr_last_error());
                    fflush(stderr);
                    _exit(1);
                }
            }
            if (rank == 0) {   // every rank has joined: the file has been read
                remove(path.c_str());
                remove((path + ".fail").c_str());
            }
        }
        // a stage: run locally, then (with a communicator) agree on every rank's outcome before the next collective
        const char* inject_stage = getenv("QASR_FAIL_STAGE");
        const int inject_rank = env_int("QASR_FAIL_RANK", -1);
        auto stage = [&](const char* what, auto&& fn) {
            std::string err;
            try {
                if (inject_stage && strcmp(inject_stage, what) == 0 && (inject_rank < 0 || inject_rank == rank))
                    throw Fail(std::string("injected failure (QASR_FAIL_STAGE=") + what + ")");
                fn();
            } catch (const std::exception& e) {
                err = e.what();
            }
            if (comm) {
                int32_t any = 0;
                ck(qasr_dist_agree(comm, err.empty() ? 0 : 1, &any), "status agreement");
                if (any) throw Fail(err.empty() ? std::string(what) + ": failed on another rank" : err);
            } else if (!err.empty()) {
                throw Fail(err);
            }
        };
        // the model: rank 0 loads / generates, the others receive it into a shell
        const char* arch = engine.c_str();
        stage("model", [&] {
            if (rank == 0)
                ck(gguf.empty() ? qasr_model_open_synthetic(arch, nullptr, 0, &model)
                                : qasr_model_open(gguf.c_str(), "hip", &model),
                   "model");
            else
                ck(qasr_model_open_shell(gguf.empty() ? nullptr : gguf.c_str(), arch, nullptr, &model), "model shell");
        });
        if (comm) {
            qasr_dist_info di;
            ck(qasr_dist_broadcast_weights(comm, model, 0, &di), "weight broadcast");
            Value b = Value::object();
            b.set("bytes", Value::integer((int64_t)di.bytes));
            b.set("ms", Value::number(di.ms));
            b.set("checksums_agree", Value::boolean(di.checksums_agree != 0));
            info.set("weight_broadcast", b);
        }
        size_t n = 0;
        std::vector<float> pcm, core;
        double t_loaded = 0;
        int64_t T = 0;
        stage("vad", [&] {
            ck(qasr_session_open(model, "f16", 32768, &sess), "session");
            if (inv) ck(qasr_session_set_batch_invariant(sess, 1), "batch invariance");
            // the recording (every rank reads it: a file, like the app's path-mode requests)
            ck(qasr_audio_load_path(wav.c_str(), nullptr, 0, &n), "audio");
            pcm.resize(std::max<size_t>(n, 1));
            ck(qasr_audio_load_path(wav.c_str(), pcm.data(), pcm.size(), &n), "audio");
            pcm.resize(n);
            t_loaded = now_ms();
            // 3. halo-sharded VAD
            ck(qasr_vad_open(nullptr, &vad), "vad");
            T = n_frames((int64_t)n);
            const int64_t f0 = T * rank / world, f1 = T * (rank + 1) / world;
            const int64_t h0 = std::max<int64_t>(0, f0 - kHalo), h1 = std::min<int64_t>(T, f1 + kHalo);
            if (f1 > f0) {
                std::vector<float> p(h1 - h0);
                size_t nf = 0;
                ck(qasr_vad_probabilities(vad, pcm.data() + h0 * kShift,
                                          (size_t)((h1 - 1) * kShift + kLen - h0 * kShift), p.data(), p.size(), &nf),
                   "vad probabilities");
                if ((int64_t)nf != h1 - h0) throw Fail("vad: frame count of the halo range");
                core.assign(p.begin() + (f0 - h0), p.begin() + (f1 - h0));
            }
        });
        std::vector<float> probs;
        if (comm) {
            std::vector<int32_t> bits(core.size()), per;
            memcpy(bits.data(), core.data(), core.size() * sizeof(float));
            const std::vector<int32_t> all = all_gather_i32(comm, bits, world, per);
            probs.resize(all.size());
            memcpy(probs.data(), all.data(), all.size() * sizeof(float));
        } else {
            probs = core;
        }
        if ((int64_t)probs.size() != T) throw Fail("vad: gathered frame count");
        // 4. segments (the reference's post-processing), LPT over the ranks; 5. this rank's share through one batch
        std::vector<qasr_segment> segs;
        size_t nseg = 0;
        std::vector<int64_t> seg_len;
        std::vector<std::vector<int>> shard;
        double t_vad = 0;
        stage("asr", [&] {
            qasr_vad_options vo;
            qasr_vad_default_options(&vo);
            segs.resize((size_t)T / 2 + 2);
            ck(qasr_vad_timestamps_from_probabilities(probs.data(), probs.size(), (int64_t)n, &vo, segs.data(),
                                                      segs.size(), &nseg),
               "segments");
            segs.resize(nseg);
            seg_len.resize(nseg);
            for (size_t i = 0; i < nseg; i++) seg_len[i] = segs[i].end - segs[i].start;
            shard = lpt_shard(seg_len, world);
            const std::vector<int>& mine = shard[rank];
            t_vad = now_ms();
            std::vector<const float*> ptrs;
            std::vector<size_t> lens;
            for (int i : mine) {
                ptrs.push_back(pcm.data() + segs[i].start);
                lens.push_back((size_t)seg_len[i]);
            }
            res.assign(mine.size(), qasr_result{});
            qasr_run_opts ro{max_new, force_tps, 0};
            if (!mine.empty())
                ck(qasr_run_batch(sess, ptrs.data(), lens.data(), (int32_t)mine.size(), &ro, res.data()), "asr batch");
        });
        const std::vector<int>& mine = shard[rank];
        const double t_asr = now_ms();
        // 6. token streams to rank 0 (every rank gets them; rank 0 prints)
        std::vector<std::vector<int32_t>> streams(nseg);
        if (comm) {
            std::vector<int32_t> lens_mine, flat_mine;
            for (auto& r : res) {
                lens_mine.push_back(r.n_tokens);
                flat_mine.insert(flat_mine.end(), r.tokens, r.tokens + r.n_tokens);
            }
            const int32_t nm = (int32_t)mine.size();
            std::vector<int32_t> rank_segs(world);
            size_t ns = 0, nt = 0;
            ck(qasr_dist_gather_tokens(comm, lens_mine.data(), nm, flat_mine.data(), rank_segs.data(), nullptr, 0,
                                       nullptr, 0, &ns, &nt),
               "token gather (sizes)");
            std::vector<int32_t> all_lens(std::max<size_t>(ns, 1)), all_tok(std::max<size_t>(nt, 1));
            ck(qasr_dist_gather_tokens(comm, lens_mine.data(), nm, flat_mine.data(), rank_segs.data(), all_lens.data(),
                                       all_lens.size(), all_tok.data(), all_tok.size(), &ns, &nt),
               "token gather");
            size_t si = 0, ti = 0;
            for (int r = 0; r < world; r++) {
                if (rank_segs[r] != (int32_t)shard[r].size()) throw Fail("token gather: segment counts disagree");
                for (int k = 0; k < rank_segs[r]; k++, si++) {
                    streams[shard[r][k]].assign(all_tok.begin() + ti, all_tok.begin() + ti + all_lens[si]);
                    ti += all_lens[si];
                }
            }
        } else {
            for (size_t k = 0; k < mine.size(); k++)
                streams[mine[k]].assign(res[k].tokens, res[k].tokens + res[k].n_tokens);
        }
        const double t_end = now_ms();
        if (rank == 0) {
            Value arr;
            arr.type = Value::Arr;
            int64_t speech = 0, ntok = 0;
            for (size_t i = 0; i < nseg; i++) {
                const std::vector<int32_t>& t = streams[i];
                size_t w = 0;
                ck(qasr_model_detokenize(model, t.data(), (int32_t)t.size(), nullptr, 0, &w), "detokenize");
                std::string raw(w, '\0');
                ck(qasr_model_detokenize(model, t.data(), (int32_t)t.size(), raw.data(), raw.size(), &w),
                   "detokenize");
                raw.resize(w);
                size_t ll = 0, tl = 0;
                ck(qasr_parse_transcript(raw.data(), raw.size(), nullptr, 0, &ll, nullptr, 0, &tl), "parse");
                std::string lang(ll, '\0'), text(tl, '\0');
                ck(qasr_parse_transcript(raw.data(), raw.size(), lang.data(), ll, &ll, text.data(), tl, &tl),
                   "parse");
                lang.resize(ll);
                text.resize(tl);
                Value sv = Value::object();
                sv.set("start", Value::integer(segs[i].start));
                sv.set("end", Value::integer(segs[i].end));
                int owner = 0;
                for (int r = 0; r < world; r++)
                    if (std::binary_search(shard[r].begin(), shard[r].end(), (int)i)) owner = r;
                sv.set("rank", Value::integer(owner));
                sv.set("language", Value::str(lang));
                sv.set("text", Value::str(text));
                Value tv;
                tv.type = Value::Arr;
                for (int32_t id : t) tv.a.push_back(Value::integer(id));
                sv.set("tokens", tv);
                arr.a.push_back(sv);
                speech += seg_len[i];
                ntok += (int64_t)t.size();
            }
            Value out = Value::object();
            out.set("engine", Value::str(engine));
            out.set("world", Value::integer(world));
            out.set("recording_s", Value::number((double)n / 16000.0));
            out.set("speech_s", Value::number((double)speech / 16000.0));
            out.set("segments_total", Value::integer((int64_t)nseg));
            out.set("segments_rank0", Value::integer((int64_t)mine.size()));
            out.set("tokens", Value::integer(ntok));
            out.set("ms_load", Value::number(t_loaded - t_start));
            out.set("ms_vad", Value::number(t_vad - t_loaded));
            out.set("ms_asr_rank0", Value::number(t_asr - t_vad));
            out.set("ms_pipeline", Value::number(t_end - t_loaded));
            out.set("rtf_inv", Value::number((double)n / 16000.0 / ((t_end - t_loaded) / 1e3)));
            out.set("batch_invariant", Value::boolean(inv));
            for (auto& kv : info.o) out.set(kv.first, kv.second);
            out.set("segments", arr);
            const std::string line = qjson::dumps(out);
            fwrite(line.data(), 1, line.size(), stdout);
            fputc('\n', stdout);
            fflush(stdout);
        }
    } catch (const std::exception& e) {
        fprintf(stderr, "engine longform (rank %d): %s\n", rank, e.what());
        rc = 1;
    }
    for (auto& r : res) qasr_result_free(&r);
    if (vad) qasr_vad_close(vad);
    if (sess) qasr_session_close(sess);
    if (model) qasr_model_close(model);
    if (comm) qasr_dist_close(comm);
    return rc;
}
