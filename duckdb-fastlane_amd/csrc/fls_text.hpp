// fls_text.hpp -- seeded TPC-H-like comment text (pool built on the host).
//
// TPC-H (spec 4.2.2.10) draws comment columns as random substrings of a text
// pool produced by a small sentence grammar; l_comment is 10..43 characters.
// This restates that scheme with the spec's word classes: a deterministic
// 8 MiB pool of grammar sentences, and comment(row) = pool[off, off + len)
// with off, len drawn from the row's random stream.  Feeds the FSST column of
// the "lineitem_full" workload.
#pragma once
#include <cstdint>
#include <string>
#include <string_view>

#include "fls_gen.hpp"

namespace fls {
namespace gen {

constexpr uint32_t S_COMMENT = 30, S_TEXT = 31;

inline const std::string &text_pool() {
    static const std::string pool = [] {
        static const char *const nouns[] = {
            "foxes", "ideas", "theodolites", "pinto beans", "instructions", "dependencies", "excuses",
            "platelets", "asymptotes", "courts", "dolphins", "multipliers", "sauternes", "warthogs", "frets",
            "dinos", "attainments", "somas", "Tiresias", "patterns", "forges", "braids", "hockey players",
            "frays", "warhorses", "dugouts", "notornis", "epitaphs", "pearls", "tithes", "waters", "orbits",
            "gifts", "sheaves", "depths", "sentiments", "decoys", "realms", "pains", "grouches", "escapades",
            "packages", "requests", "accounts", "deposits"};
        static const char *const verbs[] = {
            "sleep", "wake", "are", "cajole", "haggle", "nag", "use", "boost", "affix", "detect", "integrate",
            "maintain", "nod", "was", "lose", "sublate", "solve", "thrash", "promise", "engage", "hinder",
            "print", "x-ray", "breach", "eat", "grow", "impress", "mold", "poach", "serve", "run", "dazzle",
            "snooze", "doze", "unwind", "kindle", "play", "hang", "believe", "doubt"};
        static const char *const adjectives[] = {
            "furious", "sly", "careful", "blithe", "quick", "fluffy", "slow", "quiet", "ruthless", "thin",
            "close", "dogged", "daring", "brave", "stealthy", "permanent", "enticing", "idle", "busy",
            "regular", "final", "ironic", "even", "bold", "silent", "express", "special", "pending", "unusual"};
        static const char *const adverbs[] = {
            "sometimes", "always", "never", "furiously", "slyly", "carefully", "blithely", "quickly",
            "fluffily", "slowly", "quietly", "ruthlessly", "thinly", "closely", "doggedly", "daringly",
            "bravely", "stealthily", "permanently", "enticingly", "idly", "busily", "regularly", "finally",
            "ironically", "evenly", "boldly", "silently"};
        static const char *const preps[] = {
            "about", "above", "according to", "across", "after", "against", "along", "alongside of", "among",
            "around", "at", "atop", "before", "behind", "beneath", "beside", "besides", "between", "beyond",
            "by", "despite", "during", "except", "for", "from", "in place of", "inside", "instead of", "into",
            "near", "of", "on", "outside", "over", "past", "since", "through", "throughout", "to", "toward",
            "under", "until", "up", "upon", "without", "with", "within"};
        static const char *const aux[] = {"do", "may", "might", "shall", "will", "would", "can", "could",
                                          "should", "ought to", "must", "will have to", "shall have to",
                                          "could have to", "should have to", "must have to", "need to",
                                          "try to"};
        static const char *const terms[] = {".", ";", ":", "?", "!", "--"};
        auto pick = [](uint64_t &ctr, auto &arr) {
            const size_t n = sizeof(arr) / sizeof(arr[0]);
            return std::string_view(arr[rnd(kSeed, S_TEXT, ctr++) % n]);
        };
        auto roll = [](uint64_t &ctr, uint32_t k) { return (uint32_t)(rnd(kSeed, S_TEXT, ctr++) % k); };
        std::string s;
        s.reserve((8u << 20) + 256);
        uint64_t ctr = 0;
        while (s.size() < (8u << 20)) {
            auto noun_phrase = [&] {
                switch (roll(ctr, 4)) {
                case 0: s += pick(ctr, nouns); break;
                case 1: s += pick(ctr, adjectives); s += ' '; s += pick(ctr, nouns); break;
                case 2: s += pick(ctr, adjectives); s += ", "; s += pick(ctr, adjectives); s += ' '; s += pick(ctr, nouns); break;
                default: s += pick(ctr, adverbs); s += ' '; s += pick(ctr, adjectives); s += ' '; s += pick(ctr, nouns); break;
                }
            };
            auto verb_phrase = [&] {
                switch (roll(ctr, 4)) {
                case 0: s += pick(ctr, verbs); break;
                case 1: s += pick(ctr, aux); s += ' '; s += pick(ctr, verbs); break;
                case 2: s += pick(ctr, verbs); s += ' '; s += pick(ctr, adverbs); break;
                default: s += pick(ctr, aux); s += ' '; s += pick(ctr, verbs); s += ' '; s += pick(ctr, adverbs); break;
                }
            };
            noun_phrase();
            s += ' ';
            verb_phrase();
            if (roll(ctr, 2)) {
                s += ' ';
                s += pick(ctr, preps);
                s += " the ";
                noun_phrase();
            }
            s += pick(ctr, terms);
            s += ' ';
        }
        return s;
    }();
    return pool;
}

// l_comment of a row: 10..43 characters cut from the pool at [off, off + len)
// (host and device: the GPU check regenerates it next to the decoded column)
FLS_HD void comment_span(uint64_t seed, uint64_t row, uint64_t pool_size, uint64_t &off, uint32_t &len) {
    const uint64_t r = rnd(seed, S_COMMENT, row);
    len = 10 + (uint32_t)(r % 34);
    off = (r >> 8) % (pool_size - len);
}
inline std::string_view comment(uint64_t seed, uint64_t row) {
    const std::string &p = text_pool();
    uint64_t off;
    uint32_t len;
    comment_span(seed, row, p.size(), off, len);
    return std::string_view(p.data() + off, len);
}

}  // namespace gen
}  // namespace fls
