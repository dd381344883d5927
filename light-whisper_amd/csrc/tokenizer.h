// Byte-level BPE detokeniser (GPT-2/Qwen2 byte↔unicode map) + Qwen3-ASR output parsing
// ("language X<asr_text>text", qwen3_asr_server.py:326-327 consumes result.text / result.language).
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

namespace qasr {

struct Tokenizer {
    std::vector<std::string> pieces;   // token id → piece (GGUF tokenizer.ggml.tokens)
    std::vector<uint8_t> is_special;   // control / added tokens render literally
    // decode ids to UTF-8 bytes
    std::string decode(const int32_t* ids, int n) const;
    // UTF-8 text → ids by greedy longest match over the byte-level pieces (special tokens excluded).  Not the
    // canonical BPE merge order (the GGUF merges are not read), but every byte has a piece, so
    // decode(encode(t)) == t; used only for the opt-in hot-word context.
    std::vector<int32_t> encode(const std::string& text) const;
    // split "language X<asr_text>text" → (language, text); raw kept by the caller
    static void parse(const std::string& raw, std::string& language, std::string& text);
    // synthetic vocabulary for synthetic weights: byte tokens, letter pieces, and the special tokens
    void make_synthetic(int vocab, const int32_t* special_ids, const char* const* special_text, int n_special);
};

std::string utf8_replace_invalid(const std::string& in);

}  // namespace qasr
