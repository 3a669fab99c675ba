// Drives fls::ResidentSet (csrc/fls_resident.hpp, the HBM image budget policy)
// from a script on stdin, for tests/test_resident_budget.py (CPU only):
//   get <file> <dev> <bytes> <budget>   find or make room + insert; prints hit|new|none
//   shard <file> <dev> <lo> <hi> <budget>  the same for file bytes [lo, hi) (one
//                                        image per shard; idle overlapping ones replaced,
//                                        a held overlapping one returned: prints held)
//   hold <file> <dev> / drop <file> <dev>   a scan takes / gives back the image
//   release <dev>                        release_idle; prints the bytes freed
//   close <file>                         drop_owner (the file left the open cache)
//   lru <dev>                            evict_lru; prints 1 / 0
//   state <dev>                          prints used bytes and count
#include <cstdio>
#include <iostream>
#include <map>
#include <sstream>
#include <string>

#include "fls_resident.hpp"

struct Img {
    int file;
    static int live;
    explicit Img(int f) : file(f) { ++live; }
    ~Img() { --live; }
};
int Img::live = 0;

int main() {
    fls::ResidentSet<Img> set;
    std::map<std::pair<int, int>, std::shared_ptr<Img>> held;  // (file, dev) -> a scan's reference
    std::string line;
    while (std::getline(std::cin, line)) {
        std::istringstream in(line);
        std::string op;
        in >> op;
        if (op.empty()) continue;
        int file = 0, dev = 0;
        const void *owner = nullptr;
        auto key = [&](int f) { return reinterpret_cast<const void *>((uintptr_t)(f + 1) * 64); };
        fls::ResidentSet<Img>::Evicted ev;
        if (op == "get") {
            uint64_t bytes = 0, budget = 0;
            in >> file >> dev >> bytes >> budget;
            owner = key(file);
            if (set.find(owner, dev, 0, bytes)) {
                std::cout << "hit\n";
            } else if (set.make_room(dev, bytes, budget, ev)) {
                set.insert(owner, dev, 0, bytes, bytes, std::make_shared<Img>(file));
                std::cout << "new";
                for (auto &e : ev) std::cout << " evict" << e->file;
                std::cout << "\n";
            } else {
                std::cout << "none\n";
            }
        } else if (op == "shard") {
            uint64_t lo = 0, hi = 0, budget = 0;
            in >> file >> dev >> lo >> hi >> budget;
            owner = key(file);
            if (set.find(owner, dev, lo, hi)) {
                std::cout << "hit\n";
            } else if (set.find_held_overlap(owner, dev, lo, hi)) {
                std::cout << "held\n";
            } else {
                set.drop_overlap(owner, dev, lo, hi, ev);
                const size_t dropped = ev.size();
                ev.clear();
                if (set.make_room(dev, hi - lo, budget, ev)) {
                    set.insert(owner, dev, lo, hi, hi - lo, std::make_shared<Img>(file));
                    std::cout << "new replaced " << dropped << "\n";
                } else {
                    std::cout << "none\n";
                }
            }
        } else if (op == "hold") {
            in >> file >> dev;
            held[{file, dev}] = set.find_any(key(file), dev);
            std::cout << (held[{file, dev}] ? "held\n" : "absent\n");
        } else if (op == "drop") {
            in >> file >> dev;
            held.erase({file, dev});
            std::cout << "ok\n";
        } else if (op == "release") {
            in >> dev;
            std::cout << set.release_idle(dev, ev) << "\n";
        } else if (op == "close") {
            in >> file;
            set.drop_owner(key(file), ev);
            std::cout << ev.size() << "\n";
        } else if (op == "lru") {
            in >> dev;
            const bool b = set.evict_lru(dev, ev);
            std::cout << (b ? ev[0]->file : -1) << "\n";
        } else if (op == "state") {
            in >> dev;
            ev.clear();
            std::cout << set.used(dev) << " " << set.count(dev) << " live " << Img::live << "\n";
        } else {
            std::cout << "?\n";
        }
    }
    return 0;
}
