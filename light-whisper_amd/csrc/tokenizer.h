// Byte-level BPE detokeniser (GPT-2/Qwen2 byte↔unicode map) + Qwen3-ASR output parsing
// ("language X<asr_text>text", qwen3_asr_server.py:326-327 consumes result.text / result.language).
#pragma once
#include <stdint.h>

#include <memory>
#include <string>
#include <vector>

namespace qasr {

struct Tokenizer {
    std::vector<std::string> pieces;   // token id → piece (GGUF tokenizer.ggml.tokens)
    std::vector<uint8_t> is_special;   // control / added tokens render literally
    std::vector<std::string> merges;   // BPE merges "a b", rank = index (GGUF tokenizer.ggml.merges)
    // decode ids to UTF-8 bytes
    std::string decode(const int32_t* ids, int n) const;
    // UTF-8 text → ids, as Qwen2Tokenizer.encode(text, add_special_tokens=False) does (tokenization_qwen2.py): special
    // pieces split out whole; the Qwen2 pre-tokenizer regex (contractions, letter runs, single digits, symbol runs,
    // newline / space runs); GPT-2 byte-level alphabet; BPE merges by rank.  Text is taken as given (the reference
    // NFC-normalises first: NFC input — what keyboards produce — tokenises identically).  Without merges (synthetic
    // vocabularies): greedy longest match over the byte-level pieces.  decode(encode(t)) == t either way.
    std::vector<int32_t> encode(const std::string& text) const;
    // split "language X<asr_text>text" → (language, text); raw kept by the caller
    static void parse(const std::string& raw, std::string& language, std::string& text);
    // synthetic vocabulary for synthetic weights: byte tokens, letter pieces, and the special tokens
    void make_synthetic(int vocab, const int32_t* special_ids, const char* const* special_text, int n_special);

   private:
    struct Index;   // piece → id, merge → rank (built on first encode)
    mutable std::shared_ptr<const Index> index_;
    const Index& index() const;
    std::vector<int32_t> encode_greedy(const std::string& text) const;
    void bpe_word(const std::string& word, const Index& ix, std::vector<int32_t>& out) const;
};

std::string utf8_replace_invalid(const std::string& in);

}  // namespace qasr
