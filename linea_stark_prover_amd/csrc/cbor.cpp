// CBOR input of the trace crate: RawPermutationTrace
// (trace/src/permutation.rs:9-22) and RawLookupTrace (trace/src/lookup.rs:
// 10-44) as serde writes them through ciborium -- a map keyed by the field
// names; Vec -> array; [u8; 32] -> an array of 32 unsigned integers (serde's
// tuple form; a 32-byte byte string is accepted too); name -> text.  Words are
// big-endian and reduced with from_be_bytes_mod_order (permutation.rs:102).
// RawLookupTrace::read_file's defaults are applied: missing a_filter /
// b_filter entries are 1 (trace/src/lookup.rs:25-41).
#include <cstring>
#include <string>
#include <vector>

#include "prove_internal.hpp"


namespace lsp {
namespace {
// from_be_bytes_mod_order for 32 bytes: x < 2^256 < 8r, so at most 7
// subtractions of r give the canonical value; then into Montgomery form
Fr from_be32_mod_order(const uint8_t be[32]) {
    Fr x;
    for (int w = 0; w < 8; ++w) {
        const uint8_t* q = be + 32 - 4 * (w + 1);
        x.v[w] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
    }
    auto ge_r = [](const Fr& a) {
        for (int i = 7; i >= 0; --i) {
            if (a.v[i] != mod_word(i)) return a.v[i] > mod_word(i);
        }
        return true;
    };
    while (ge_r(x)) {
        uint64_t borrow = 0;
        for (int i = 0; i < 8; ++i) {
            const uint64_t d = (uint64_t)x.v[i] - mod_word(i) - borrow;
            x.v[i] = (uint32_t)d;
            borrow = (d >> 32) & 1;
        }
    }
    return fr_from_canonical(x);
}

struct Cbor {
    const uint8_t* p;
    const uint8_t* end;

    [[noreturn]] void fail(const char* what) { throw LspError(LSP_E_ARG, std::string("CBOR: ") + what); }
    uint8_t byte() {
        if (p >= end) fail("truncated input");
        return *p++;
    }
    // major type, argument; `indef` set for an indefinite-length item
    uint64_t head(int& major, bool& indef) {
        const uint8_t ib = byte();
        major = ib >> 5;
        const int ai = ib & 31;
        indef = false;
        if (ai < 24) return (uint64_t)ai;
        if (ai == 31) {
            if (major < 2 || major > 5) fail("indefinite length on a non-container");
            indef = true;
            return 0;
        }
        int n = ai == 24 ? 1 : ai == 25 ? 2 : ai == 26 ? 4 : ai == 27 ? 8 : 0;
        if (!n) fail("reserved additional information");
        uint64_t v = 0;
        for (int i = 0; i < n; ++i) v = (v << 8) | byte();
        return v;
    }
    bool at_break() { return p < end && *p == 0xff; }
    void skip_tags(int& major, uint64_t& arg, bool& indef) {
        while (major == 6) arg = head(major, indef);
    }
    uint64_t uint_item() {
        int m;
        bool ind;
        uint64_t v = head(m, ind);
        skip_tags(m, v, ind);
        if (m != 0) fail("expected an unsigned integer");
        return v;
    }
    std::string text() {
        int m;
        bool ind;
        uint64_t n = head(m, ind);
        skip_tags(m, n, ind);
        if (m != 3) fail("expected a text string");
        std::string s;
        if (ind) {
            while (!at_break()) s += text();
            ++p;
            return s;
        }
        if ((uint64_t)(end - p) < n) fail("truncated text");
        s.assign((const char*)p, n);
        p += n;
        return s;
    }
    void skip() {
        int m;
        bool ind;
        uint64_t n = head(m, ind);
        skip_tags(m, n, ind);
        if (m == 2 || m == 3) {
            if (ind) {
                while (!at_break()) skip();
                ++p;
            } else {
                if ((uint64_t)(end - p) < n) fail("truncated string");
                p += n;
            }
        } else if (m == 4 || m == 5) {
            const uint64_t k = m == 5 ? 2 : 1;
            if (ind) {
                while (!at_break()) skip();
                ++p;
            } else {
                for (uint64_t i = 0; i < n * k; ++i) skip();
            }
        }
    }
    // array header: returns the count, or UINT64_MAX for indefinite
    uint64_t array() {
        int m;
        bool ind;
        uint64_t n = head(m, ind);
        skip_tags(m, n, ind);
        if (m != 4) fail("expected an array");
        return ind ? UINT64_MAX : n;
    }
    bool more(uint64_t n, uint64_t i) {
        if (n != UINT64_MAX) return i < n;
        if (at_break()) {
            ++p;
            return false;
        }
        return true;
    }
    // [u8; 32] (array of 32 uints or a 32-byte byte string) -> Fr via from_be_bytes_mod_order
    Fr word() {
        uint8_t be[32];
        int m;
        bool ind;
        const uint8_t* save = p;
        uint64_t n = head(m, ind);
        skip_tags(m, n, ind);
        if (m == 2 && !ind) {
            if (n != 32) fail("a word must be 32 bytes");
            if ((uint64_t)(end - p) < 32) fail("truncated word");
            std::memcpy(be, p, 32);
            p += 32;
        } else if (m == 4) {
            p = save;
            const uint64_t k = array();
            uint64_t i = 0;
            for (; more(k, i); ++i) {
                if (i >= 32) fail("a word must have 32 bytes");
                const uint64_t v = uint_item();
                if (v > 255) fail("a word byte exceeds 255");
                be[i] = (uint8_t)v;
            }
            if (i != 32) fail("a word must have 32 bytes");
        } else {
            fail("expected a 32-byte word");
        }
        return from_be32_mod_order(be);
    }
    // item kind at the cursor without consuming it: 0 uint, 2 bytes, 4 array, other major
    int peek_major() {
        Cbor q = *this;
        int m;
        bool ind;
        uint64_t n = q.head(m, ind);
        q.skip_tags(m, n, ind);
        return m;
    }
    // is the array at the cursor [[[word]]] (a lookup's tables) rather than [[word]]?
    bool b_is_nested() {
        Cbor q = *this;
        const uint64_t n1 = q.array();
        if (!q.more(n1, 0) || q.peek_major() != 4) return false;
        const uint64_t n2 = q.array();  // b[0]: a column (of words) or a table (of columns)
        if (!q.more(n2, 0)) return false;
        if (q.peek_major() == 2) return false;  // b[0][0] is a byte-string word
        if (q.peek_major() != 4) return false;
        q.array();  // b[0][0]: a word (array of uints) or a column (array of words)
        if (q.at_break() || q.p >= q.end) return false;
        const int m = q.peek_major();
        return m == 4 || m == 2;
    }
    std::vector<Fr> column() {
        std::vector<Fr> c;
        const uint64_t n = array();
        for (uint64_t i = 0; more(n, i); ++i) c.push_back(word());
        return c;
    }
    std::vector<std::vector<Fr>> columns() {
        std::vector<std::vector<Fr>> cs;
        const uint64_t n = array();
        for (uint64_t i = 0; more(n, i); ++i) cs.push_back(column());
        return cs;
    }
};
}  // namespace

lsp_raw_trace* parse_raw_trace(const uint8_t* buf, size_t len) {
    Cbor c{buf, buf + len};
    int m;
    bool ind;
    uint64_t n = c.head(m, ind);
    c.skip_tags(m, n, ind);
    if (m != 5) c.fail("a trace is a map of its fields");
    auto t = std::make_unique<lsp_raw_trace>();
    bool has_a = false, has_b = false, lookup_fields = false, nested_b = false;
    std::vector<std::vector<std::vector<Fr>>> tables;
    for (uint64_t i = 0; c.more(ind ? UINT64_MAX : n, i); ++i) {
        const std::string key = c.text();
        if (key == "a") {
            t->a = c.columns();
            has_a = true;
        } else if (key == "b") {
            // permutation: [[word]]; lookup: [[[word]]]
            if (c.b_is_nested()) {
                const uint64_t nt = c.array();
                for (uint64_t j = 0; c.more(nt, j); ++j) tables.push_back(c.columns());
                nested_b = true;
            } else {
                t->b = c.columns();
            }
            has_b = true;
        } else if (key == "name") {
            t->name = c.text();
        } else if (key == "a_filter") {
            t->a_filter = c.column();
            lookup_fields = true;
        } else if (key == "b_filter") {
            t->b_filter = c.columns();
            lookup_fields = true;
        } else {
            c.skip();
        }
    }
    if (!has_a || !has_b || t->a.empty()) c.fail("a trace needs non-empty 'a' and 'b'");
    if (nested_b || lookup_fields) {
        t->kind = LSP_AIR_LOOKUP;
        if (!nested_b) {  // an empty b or a flat b in a lookup: one table per column is not the format
            if (!t->b.empty()) c.fail("lookup 'b' must be a list of tables");
        }
        if (tables.empty()) c.fail("a lookup needs at least one B table");
        t->ntables = (uint32_t)tables.size();
        t->nbc = (uint32_t)tables[0].size();
        for (auto& tab : tables) {
            if (tab.size() != t->nbc) c.fail("all B tables must have the same number of columns");
            for (auto& col : tab) t->b.push_back(std::move(col));
        }
        // read_file: pad the filters with 1 (enabled)
        const Fr one = fr_one();
        while (t->a_filter.size() < t->a[0].size()) t->a_filter.push_back(one);
        while (t->b_filter.size() < t->ntables) t->b_filter.emplace_back();
        for (uint32_t j = 0; j < t->ntables; ++j)
            while (t->b_filter[j].size() < t->b[(size_t)j * t->nbc].size()) t->b_filter[j].push_back(one);
    } else {
        t->kind = LSP_AIR_PERMUTATION;
        t->ntables = (uint32_t)t->b.size();
    }
    if (c.p != c.end) c.fail("trailing bytes after the trace");
    return t.release();
}

// the largest column length (get_max_height) and the block width
void raw_trace_shape(const lsp_raw_trace& t, size_t& height, size_t& width) {
    height = 0;
    for (auto& c : t.a) height = std::max(height, c.size());
    for (auto& c : t.b) height = std::max(height, c.size());
    if (t.kind == LSP_AIR_LOOKUP)
        width = t.a.size() + (size_t)t.ntables * (t.nbc + 3) + 3;
    else
        width = t.a.size() + t.b.size() + 2;
}

// the columns resized to `height` (Vec::resize with zero words), column-major:
// a.., b.. (lookup: table-major), then for a lookup a_filter, b_filters..
std::vector<Fr> raw_trace_columns(const lsp_raw_trace& t, size_t height) {
    std::vector<Fr> out;
    auto put = [&](const std::vector<Fr>& c) {
        LSP_REQUIRE(c.size() <= height, LSP_E_ARG, "column longer than the requested height");
        out.insert(out.end(), c.begin(), c.end());
        out.resize(out.size() + (height - c.size()), fr_zero());
    };
    for (auto& c : t.a) put(c);
    for (auto& c : t.b) put(c);
    if (t.kind == LSP_AIR_LOOKUP) {
        put(t.a_filter);
        for (auto& f : t.b_filter) put(f);
    }
    return out;
}

}  // namespace lsp
