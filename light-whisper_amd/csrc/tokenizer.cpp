#include "tokenizer.h"

#include <string.h>

#include <algorithm>
#include <unordered_map>

#include "common.h"

namespace qasr {

namespace {
// GPT-2 bytes_to_unicode inverse: codepoint → byte (-1 if not a byte codepoint)
struct ByteMap {
    int cp2byte[512];
    int byte2cp[256];
    ByteMap() {
        for (int i = 0; i < 512; i++) cp2byte[i] = -1;
        int n = 0;
        for (int b = 0; b < 256; b++) {
            bool keep = (b >= '!' && b <= '~') || (b >= 0xA1 && b <= 0xAC) || (b >= 0xAE && b <= 0xFF);
            int cp = keep ? b : 256 + n++;
            byte2cp[b] = cp;
            cp2byte[cp] = b;
        }
    }
};
const ByteMap& bmap() {
    static ByteMap m;
    return m;
}

void append_utf8(std::string& s, int cp) {
    if (cp < 0x80) s += (char)cp;
    else if (cp < 0x800) {
        s += (char)(0xC0 | (cp >> 6));
        s += (char)(0x80 | (cp & 0x3F));
    } else {
        s += (char)(0xE0 | (cp >> 12));
        s += (char)(0x80 | ((cp >> 6) & 0x3F));
        s += (char)(0x80 | (cp & 0x3F));
    }
}
}  // namespace

// bytes → valid UTF-8 the way Python's bytes.decode("utf-8", errors="replace") does it (the Qwen2 byte-level BPE
// tokenizer's decode, errors="replace"): each maximal ill-formed subpart becomes one U+FFFD
std::string utf8_replace_invalid(const std::string& in) {
    const unsigned char* s = (const unsigned char*)in.data();
    const size_t n = in.size();
    std::string out;
    out.reserve(n);
    size_t i = 0;
    while (i < n) {
        const unsigned c = s[i];
        if (c < 0x80) {
            out += (char)c;
            i++;
            continue;
        }
        int len = 0;
        unsigned lo = 0x80, hi = 0xBF;   // allowed range of the second byte
        if (c >= 0xC2 && c <= 0xDF) len = 2;
        else if (c == 0xE0) len = 3, lo = 0xA0;
        else if ((c >= 0xE1 && c <= 0xEC) || c == 0xEE || c == 0xEF) len = 3;
        else if (c == 0xED) len = 3, hi = 0x9F;
        else if (c == 0xF0) len = 4, lo = 0x90;
        else if (c >= 0xF1 && c <= 0xF3) len = 4;
        else if (c == 0xF4) len = 4, hi = 0x8F;
        int ok = 1;   // bytes of the sequence accepted so far
        if (len > 0) {
            for (; ok < len && i + ok < n; ok++) {
                const unsigned b = s[i + ok];
                const bool good = ok == 1 ? (b >= lo && b <= hi) : (b >= 0x80 && b <= 0xBF);
                if (!good) break;
            }
        }
        if (len > 0 && ok == len) {
            out.append((const char*)s + i, (size_t)len);
            i += (size_t)len;
        } else {
            out += "\xEF\xBF\xBD";
            i += (size_t)ok;
        }
    }
    return out;
}

std::string Tokenizer::decode(const int32_t* ids, int n) const {
    const ByteMap& bm = bmap();
    std::string out;
    for (int i = 0; i < n; i++) {
        const int id = ids[i];
        if (id < 0 || id >= (int)pieces.size()) continue;
        const std::string& p = pieces[id];
        if (!is_special.empty() && is_special[id]) {
            out += p;
            continue;
        }
        // walk UTF-8 codepoints; byte codepoints map back to raw bytes
        const unsigned char* s = (const unsigned char*)p.data();
        size_t k = 0;
        while (k < p.size()) {
            int cp, len;
            if (s[k] < 0x80) { cp = s[k]; len = 1; }
            else if ((s[k] & 0xE0) == 0xC0 && k + 1 < p.size()) { cp = ((s[k] & 0x1F) << 6) | (s[k + 1] & 0x3F); len = 2; }
            else if ((s[k] & 0xF0) == 0xE0 && k + 2 < p.size()) {
                cp = ((s[k] & 0x0F) << 12) | ((s[k + 1] & 0x3F) << 6) | (s[k + 2] & 0x3F);
                len = 3;
            } else { cp = -1; len = 1; }
            if (cp >= 0 && cp < 512 && bm.cp2byte[cp] >= 0) out += (char)bm.cp2byte[cp];
            else out.append((const char*)s + k, (size_t)len);
            k += (size_t)len;
        }
    }
    return utf8_replace_invalid(out);
}

void Tokenizer::parse(const std::string& raw, std::string& language, std::string& text) {
    static const char* tag = "<asr_text>";
    size_t at = raw.find(tag);
    if (at == std::string::npos) {
        language.clear();
        text = raw;
        return;
    }
    std::string head = raw.substr(0, at);
    text = raw.substr(at + strlen(tag));
    const std::string pre = "language ";
    size_t p = head.find(pre);
    language = p == std::string::npos ? head : head.substr(p + pre.size());
    // trim
    while (!language.empty() && (language.back() == ' ' || language.back() == '\n')) language.pop_back();
    while (!language.empty() && (language[0] == ' ' || language[0] == '\n')) language.erase(0, 1);
    if (language == "None") language.clear();
}

std::vector<int32_t> Tokenizer::encode(const std::string& text) const {
    const ByteMap& bm = bmap();
    std::unordered_map<std::string, int32_t> index;
    size_t maxlen = 1;
    for (int32_t id = 0; id < (int32_t)pieces.size(); id++) {
        if (!is_special.empty() && is_special[id]) continue;
        if (pieces[id].empty()) continue;
        index.emplace(pieces[id], id);   // first id wins for duplicate pieces
        maxlen = std::max(maxlen, pieces[id].size());
    }
    std::string u;   // the text in the byte-level alphabet (each byte one codepoint, 1-2 UTF-8 bytes)
    for (unsigned char c : text) append_utf8(u, bm.byte2cp[c]);
    std::vector<int32_t> out;
    size_t i = 0;
    while (i < u.size()) {
        size_t best = 0;
        int32_t best_id = -1;
        for (size_t L = std::min(maxlen, u.size() - i); L >= 1; L--) {
            if (i + L < u.size() && ((unsigned char)u[i + L] & 0xC0) == 0x80) continue;   // codepoint boundary
            auto it = index.find(u.substr(i, L));
            if (it != index.end()) {
                best = L;
                best_id = it->second;
                break;
            }
        }
        QASR_CHECK(best_id >= 0, QASR_E_FORMAT, "tokenizer: byte without a piece");
        out.push_back(best_id);
        i += best;
    }
    return out;
}

void Tokenizer::make_synthetic(int vocab, const int32_t* special_ids, const char* const* special_text, int n_special) {
    const ByteMap& bm = bmap();
    pieces.assign(vocab, std::string());
    is_special.assign(vocab, 0);
    for (int id = 0; id < vocab; id++) {
        std::string s;
        if (id < 256) {
            append_utf8(s, bm.byte2cp[id]);
        } else {
            // 1-4 lowercase letters, optionally with a leading 'Ġ' (byte-level space), from a hash of the id
            uint64_t h = smix(0x5eedULL ^ (uint64_t)id);
            int len = 1 + (int)(h & 3);
            if ((h >> 2) & 1) append_utf8(s, bm.byte2cp[' ']);
            for (int j = 0; j < len; j++) s += (char)('a' + (int)((h >> (8 + 5 * j)) % 26));
        }
        pieces[id] = s;
    }
    for (int i = 0; i < n_special; i++) {
        int id = special_ids[i];
        if (id >= 0 && id < vocab) {
            pieces[id] = special_text[i];
            is_special[id] = 1;
        }
    }
}

}  // namespace qasr
