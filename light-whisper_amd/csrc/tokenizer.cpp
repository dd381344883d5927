#include "tokenizer.h"

#include <string.h>

#include <algorithm>
#include <climits>
#include <mutex>
#include <unordered_map>

#include "common.h"
#include "unicode_ranges.h"

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

namespace {
// UTF-8 ↔ codepoints (the decoder's output is valid UTF-8: it went through utf8_replace_invalid)
std::u32string to_u32(const std::string& s) {
    std::u32string o;
    const unsigned char* p = (const unsigned char*)s.data();
    for (size_t i = 0; i < s.size();) {
        const unsigned c = p[i];
        int len = c < 0x80 ? 1 : c < 0xE0 ? 2 : c < 0xF0 ? 3 : 4;
        if (i + len > s.size()) len = 1;
        char32_t cp = len == 1 ? c : len == 2 ? c & 0x1F : len == 3 ? c & 0x0F : c & 0x07;
        for (int k = 1; k < len; k++) cp = (cp << 6) | (p[i + k] & 0x3F);
        o += cp;
        i += (size_t)len;
    }
    return o;
}
std::string to_utf8(const std::u32string& s) {
    std::string o;
    for (char32_t c : s) {
        if (c < 0x80) o += (char)c;
        else if (c < 0x800) o += (char)(0xC0 | (c >> 6)), o += (char)(0x80 | (c & 0x3F));
        else if (c < 0x10000)
            o += (char)(0xE0 | (c >> 12)), o += (char)(0x80 | ((c >> 6) & 0x3F)), o += (char)(0x80 | (c & 0x3F));
        else
            o += (char)(0xF0 | (c >> 18)), o += (char)(0x80 | ((c >> 12) & 0x3F)), o += (char)(0x80 | ((c >> 6) & 0x3F)),
                o += (char)(0x80 | (c & 0x3F));
    }
    return o;
}
// Python str.isspace / str.strip() / str.splitlines() separators / ASCII str.lower()
bool py_space(char32_t c) {
    return (c >= 0x09 && c <= 0x0D) || (c >= 0x1C && c <= 0x20) || c == 0x85 || c == 0xA0 || c == 0x1680 ||
           (c >= 0x2000 && c <= 0x200A) || c == 0x2028 || c == 0x2029 || c == 0x202F || c == 0x205F || c == 0x3000;
}
bool py_linebreak(char32_t c) {
    return c == 0x0A || c == 0x0B || c == 0x0C || c == 0x0D || c == 0x1C || c == 0x1D || c == 0x1E || c == 0x85 ||
           c == 0x2028 || c == 0x2029;
}
std::u32string strip(const std::u32string& s) {
    size_t b = 0, e = s.size();
    while (b < e && py_space(s[b])) b++;
    while (e > b && py_space(s[e - 1])) e--;
    return s.substr(b, e - b);
}
std::u32string lower_ascii(std::u32string s) {
    for (auto& c : s)
        if (c >= 'A' && c <= 'Z') c += 32;
    return s;
}

// _detect_and_fix_repetitions (processing_qwen3_asr.py:310-380, threshold 20): runs of > 20 equal characters
// collapse to one, then the first pattern of 1-20 characters repeated ≥ 20 times collapses to one copy (and the
// rest of the string is fixed the same way)
std::u32string fix_char_repeats(const std::u32string& s, size_t th) {
    std::u32string r;
    for (size_t i = 0; i < s.size();) {
        size_t cnt = 1;
        while (i + cnt < s.size() && s[i + cnt] == s[i]) cnt++;
        if (cnt > th) r += s[i];
        else r.append(s, i, cnt);
        i += cnt;
    }
    return r;
}
std::u32string fix_pattern_repeats(const std::u32string& s, int64_t th, int64_t max_len = 20) {
    const int64_t n = (int64_t)s.size(), min_rep = th * 2;
    if (n < min_rep) return s;
    std::u32string r;
    int64_t i = 0;
    bool found = false;
    while (i <= n - min_rep) {
        found = false;
        for (int64_t k = 1; k <= max_len; k++) {
            if (i + k * th > n) break;
            bool valid = true;
            for (int64_t rep = 1; rep < th && valid; rep++) valid = s.compare((size_t)(i + rep * k), (size_t)k, s, (size_t)i, (size_t)k) == 0;
            if (valid) {
                int64_t end = i + th * k;
                while (end + k <= n && s.compare((size_t)end, (size_t)k, s, (size_t)i, (size_t)k) == 0) end += k;
                r.append(s, (size_t)i, (size_t)k);
                r += fix_pattern_repeats(s.substr((size_t)end), th, max_len);
                i = n;
                found = true;
                break;
            }
        }
        if (found) break;
        r += s[(size_t)i];
        i++;
    }
    if (!found) r.append(s, (size_t)std::min(i, n), std::u32string::npos);
    return r;
}
}  // namespace

// Qwen3-ASR output → (language, transcription).  transcribe.cpp's own parser is not available (third-party, absent:
// SURVEY §8(c)); this restates the in-container Qwen3-ASR reference parser _parse_single_output
// (transformers/models/qwen3_asr/processing_qwen3_asr.py:159-196, "like the original implementation"): strip, keep
// what follows "assistant\n", the repetition fix, split at the first "<asr_text>" (none: all of it is the text, no
// language), "language none" (any case) → no language, else the first non-empty line of the prefix with its
// "language " prefix (any case) removed.  "" = no language (the server then reports "unknown",
// qwen3_asr_server.py:327).  Lower-casing is ASCII-only.
void Tokenizer::parse(const std::string& raw, std::string& language, std::string& text) {
    language.clear();
    text.clear();
    std::u32string t = strip(to_u32(raw));
    if (t.empty()) return;
    static const std::u32string kAssistant = U"assistant\n", kMarker = U"<asr_text>", kLang = U"language ";
    if (size_t a = t.find(kAssistant); a != std::u32string::npos) t = t.substr(a + kAssistant.size());
    t = fix_pattern_repeats(fix_char_repeats(t, 20), 20);
    const size_t at = t.find(kMarker);
    if (at == std::u32string::npos) {
        text = to_utf8(strip(t));
        return;
    }
    const std::u32string prefix = strip(t.substr(0, at));
    text = to_utf8(strip(t.substr(at + kMarker.size())));
    if (lower_ascii(prefix) == U"language none") return;
    for (size_t b = 0; b < prefix.size();) {
        size_t e = b;
        while (e < prefix.size() && !py_linebreak(prefix[e])) e++;
        const std::u32string line = strip(prefix.substr(b, e - b));
        b = e + (e < prefix.size() && prefix[e] == 0x0D && e + 1 < prefix.size() && prefix[e + 1] == 0x0A ? 2 : 1);
        if (line.empty()) continue;
        if (lower_ascii(line).compare(0, kLang.size(), kLang) == 0) language = to_utf8(strip(line.substr(kLang.size())));
        else language = to_utf8(line);
        break;
    }
}

std::vector<int32_t> Tokenizer::encode_greedy(const std::string& text) const {
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

struct Tokenizer::Index {
    std::unordered_map<std::string, int32_t> piece;   // non-special pieces (first id wins)
    std::unordered_map<std::string, int> rank;        // "a b" → merge rank
    std::vector<std::pair<std::string, int32_t>> special;   // special pieces, longest first
};

const Tokenizer::Index& Tokenizer::index() const {
    static std::mutex mu;   // a model's tokenizer is shared by its sessions' threads
    std::lock_guard<std::mutex> lock(mu);
    if (index_) return *index_;
    auto ix = std::make_shared<Index>();
    for (int32_t id = 0; id < (int32_t)pieces.size(); id++) {
        if (pieces[id].empty()) continue;
        if (!is_special.empty() && is_special[id]) ix->special.emplace_back(pieces[id], id);
        else ix->piece.emplace(pieces[id], id);
    }
    std::stable_sort(ix->special.begin(), ix->special.end(),
                     [](const auto& a, const auto& b) { return a.first.size() > b.first.size(); });
    for (int r = 0; r < (int)merges.size(); r++) ix->rank.emplace(merges[r], r);
    index_ = ix;
    return *index_;
}

namespace {
bool in_ranges(const UniRange* r, size_t n, char32_t c) {
    size_t lo = 0, hi = n;
    while (lo < hi) {
        const size_t mid = (lo + hi) / 2;
        if (c < r[mid].lo) hi = mid;
        else if (c > r[mid].hi) lo = mid + 1;
        else return true;
    }
    return false;
}
bool uni_L(char32_t c) { return in_ranges(kUniLetter, sizeof kUniLetter / sizeof kUniLetter[0], c); }
bool uni_N(char32_t c) { return in_ranges(kUniNumber, sizeof kUniNumber / sizeof kUniNumber[0], c); }
// \s of the regex engines (the Unicode White_Space property)
bool uni_ws(char32_t c) {
    return (c >= 0x09 && c <= 0x0D) || c == 0x20 || c == 0x85 || c == 0xA0 || c == 0x1680 || (c >= 0x2000 && c <= 0x200A) ||
           c == 0x2028 || c == 0x2029 || c == 0x202F || c == 0x205F || c == 0x3000;
}
bool uni_nl(char32_t c) { return c == '\r' || c == '\n'; }
char32_t lower1(char32_t c) { return c >= 'A' && c <= 'Z' ? c + 32 : c; }

// length of the Qwen2 pre-tokenizer match at i (tokenization_qwen2.py PRETOKENIZE_REGEX, alternatives in order):
//   (?i:'s|'t|'re|'ve|'m|'ll|'d) | [^\r\n\p{L}\p{N}]?\p{L}+ | \p{N} | ?[^\s\p{L}\p{N}]+[\r\n]* | \s*[\r\n]+ |
//   \s+(?!\S) | \s+
size_t pretoken(const std::u32string& c, size_t i) {
    const size_t n = c.size();
    if (c[i] == '\'' && i + 1 < n) {
        const char32_t a = lower1(c[i + 1]);
        if (a == 's' || a == 't' || a == 'm' || a == 'd') return 2;
        if (i + 2 < n) {
            const char32_t b = lower1(c[i + 2]);
            if ((a == 'r' && b == 'e') || (a == 'v' && b == 'e') || (a == 'l' && b == 'l')) return 3;
        }
    }
    auto other = [](char32_t x) { return !uni_ws(x) && !uni_L(x) && !uni_N(x); };
    {
        size_t j = i;
        if (!uni_nl(c[j]) && !uni_L(c[j]) && !uni_N(c[j]) && j + 1 < n && uni_L(c[j + 1])) j++;
        if (uni_L(c[j])) {
            while (j < n && uni_L(c[j])) j++;
            return j - i;
        }
    }
    if (uni_N(c[i])) return 1;
    {
        size_t j = i;
        if (c[j] == ' ' && j + 1 < n && other(c[j + 1])) j++;
        if (other(c[j])) {
            while (j < n && other(c[j])) j++;
            while (j < n && uni_nl(c[j])) j++;
            return j - i;
        }
    }
    if (uni_ws(c[i])) {
        size_t j = i;
        while (j < n && uni_ws(c[j])) j++;
        for (size_t k = j; k > i; k--)
            if (uni_nl(c[k - 1])) return k - i;    // \s*[\r\n]+: up to the run's last newline
        if (j == n) return j - i;                  // \s+(?!\S)
        if (j - i >= 2) return j - i - 1;          //   (leaving the last space to the next token)
        return j - i;                              // \s+
    }
    return 1;
}
}  // namespace

// BPE of one pre-token (byte-level symbols), merges by rank (lowest first, every occurrence left to right)
void Tokenizer::bpe_word(const std::string& word, const Index& ix, std::vector<int32_t>& out) const {
    const ByteMap& bm = bmap();
    std::vector<std::string> sym;
    for (unsigned char ch : word) {
        std::string u;
        append_utf8(u, bm.byte2cp[ch]);
        sym.push_back(u);
    }
    while (sym.size() > 1) {
        int best = INT32_MAX;
        size_t at = 0;
        for (size_t k = 0; k + 1 < sym.size(); k++) {
            auto it = ix.rank.find(sym[k] + " " + sym[k + 1]);
            if (it != ix.rank.end() && it->second < best) best = it->second, at = k;
        }
        if (best == INT32_MAX) break;
        const std::string a = sym[at], b = sym[at + 1];
        std::vector<std::string> nw;
        for (size_t k = 0; k < sym.size();) {
            if (k + 1 < sym.size() && sym[k] == a && sym[k + 1] == b) {
                nw.push_back(a + b);
                k += 2;
            } else {
                nw.push_back(sym[k++]);
            }
        }
        sym.swap(nw);
    }
    for (const std::string& x : sym) {
        auto it = ix.piece.find(x);
        QASR_CHECK(it != ix.piece.end(), QASR_E_FORMAT, "tokenizer: BPE symbol without a piece");
        out.push_back(it->second);
    }
}

std::vector<int32_t> Tokenizer::encode(const std::string& text) const {
    if (merges.empty()) return encode_greedy(text);
    const Index& ix = index();
    std::vector<int32_t> out;
    size_t pos = 0;
    while (pos < text.size()) {
        // the next special piece (added tokens are matched before the pre-tokenizer)
        size_t sp_at = std::string::npos;
        const std::pair<std::string, int32_t>* sp = nullptr;
        for (const auto& s : ix.special) {
            const size_t f = text.find(s.first, pos);
            if (f != std::string::npos && (f < sp_at)) sp_at = f, sp = &s;
        }
        const size_t end = sp ? sp_at : text.size();
        const std::u32string c = to_u32(text.substr(pos, end - pos));
        for (size_t i = 0; i < c.size();) {
            const size_t len = pretoken(c, i);
            bpe_word(to_utf8(c.substr(i, len)), ix, out);
            i += len;
        }
        if (!sp) break;
        out.push_back(sp->second);
        pos = sp_at + sp->first.size();
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
