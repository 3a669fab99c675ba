// fls_resident.hpp -- the process-wide byte budget of HBM-resident file images.
//
// The scan pipeline keeps a scanned file's compressed bytes in HBM so a warm
// query moves only decoded bytes over PCIe (flsgpu.hip, resident_image).  The
// reference holds nothing between queries (its closeFile releases everything,
// src/fastlanes_facade.cpp:202-210), so this cache must never crowd out the
// allocations a scan needs: one byte budget per GPU over every cached image,
// least recently used images evicted first, never an image a running scan
// uses, and everything idle released on demand (fls_release_device_memory).
//
// This header is the policy only -- no HIP -- so the CPU tests compile and
// drive it directly (tests/test_resident_budget.py).  Img is the image type
// (flsgpu.hip: DevImage); an image is "in use" while anyone besides this set
// holds its shared_ptr (a scan's ScanDev::dimg).  The caller serialises every
// call (one mutex) and frees the evicted images it is handed (flsgpu.hip does
// so under that mutex, before it allocates the image they made room for).
#pragma once
#include <algorithm>
#include <cstdint>
#include <memory>
#include <vector>

namespace fls {

template <class Img>
class ResidentSet {
  public:
    struct Entry {
        const void *owner;   // the mapped file the image belongs to
        int dev;
        uint64_t lo, hi;     // file byte range the image holds
        uint64_t bytes;      // device bytes allocated for it
        uint64_t tick;       // last use
        std::shared_ptr<Img> img;
    };
    using Evicted = std::vector<std::shared_ptr<Img>>;

    // owner's image on dev that holds the file bytes [lo, hi), if any (a use:
    // it becomes the most recent).  One file may have several images on one
    // GPU: one per shard when a connection lists the GPU more than once (the
    // 8-way split rehearsed on one GPU).
    std::shared_ptr<Img> find(const void *owner, int dev, uint64_t lo, uint64_t hi) {
        for (Entry &e : e_)
            if (e.owner == owner && e.dev == dev && e.lo <= lo && hi <= e.hi) {
                e.tick = ++tick_;
                return e.img;
            }
        return nullptr;
    }
    // any image of owner on dev (a scan's hold in the CPU driver)
    std::shared_ptr<Img> find_any(const void *owner, int dev) {
        for (Entry &e : e_)
            if (e.owner == owner && e.dev == dev) {
                e.tick = ++tick_;
                return e.img;
            }
        return nullptr;
    }
    // an image of owner on dev overlapping [lo, hi) that a scan holds (made
    // for another split of the table: the caller decodes what it covers and
    // streams the rest), or none
    std::shared_ptr<Img> find_held_overlap(const void *owner, int dev, uint64_t lo, uint64_t hi) {
        for (Entry &e : e_)
            if (e.owner == owner && e.dev == dev && e.lo < hi && lo < e.hi && !idle(e)) {
                e.tick = ++tick_;
                return e.img;
            }
        return nullptr;
    }
    uint64_t used(int dev) const {
        uint64_t t = 0;
        for (const Entry &e : e_)
            if (dev < 0 || e.dev == dev) t += e.bytes;
        return t;
    }
    size_t count(int dev) const {
        size_t n = 0;
        for (const Entry &e : e_) n += dev < 0 || e.dev == dev;
        return n;
    }
    static bool idle(const Entry &e) { return e.img.use_count() == 1; }
    // Evict idle images of dev, least recently used first, until need more
    // bytes fit under budget; the evicted images go to out.  False when even
    // evicting every idle image would not make room (nothing is evicted then).
    bool make_room(int dev, uint64_t need, uint64_t budget, Evicted &out) {
        if (need > budget) return false;
        uint64_t u = used(dev), freeable = 0;
        for (const Entry &e : e_)
            if (e.dev == dev && idle(e)) freeable += e.bytes;
        if (u + need > budget && u - freeable + need > budget) return false;
        while (u + need > budget) {
            size_t v = e_.size();
            for (size_t i = 0; i < e_.size(); ++i)
                if (e_[i].dev == dev && idle(e_[i]) && (v == e_.size() || e_[i].tick < e_[v].tick)) v = i;
            if (v == e_.size()) return false;  // (not reached: freeable covered it)
            u -= e_[v].bytes;
            out.push_back(std::move(e_[v].img));
            e_.erase(e_.begin() + (long)v);
        }
        return true;
    }
    void insert(const void *owner, int dev, uint64_t lo, uint64_t hi, uint64_t bytes, std::shared_ptr<Img> img) {
        e_.push_back(Entry{owner, dev, lo, hi, bytes, ++tick_, std::move(img)});
    }
    // every image of owner (a file leaving the open cache), in use or not: a
    // scan holding one keeps it alive through its own reference
    void drop_owner(const void *owner, Evicted &out) {
        for (size_t i = e_.size(); i-- > 0;)
            if (e_[i].owner == owner) {
                out.push_back(std::move(e_[i].img));
                e_.erase(e_.begin() + (long)i);
            }
    }
    // owner's idle images on dev overlapping [lo, hi) (replaced: made for
    // another split of the table)
    void drop_overlap(const void *owner, int dev, uint64_t lo, uint64_t hi, Evicted &out) {
        for (size_t i = e_.size(); i-- > 0;)
            if (e_[i].owner == owner && e_[i].dev == dev && e_[i].lo < hi && lo < e_[i].hi && idle(e_[i])) {
                out.push_back(std::move(e_[i].img));
                e_.erase(e_.begin() + (long)i);
            }
    }
    // the least recently used idle image of dev; false when there is none
    bool evict_lru(int dev, Evicted &out) {
        size_t v = e_.size();
        for (size_t i = 0; i < e_.size(); ++i)
            if (e_[i].dev == dev && idle(e_[i]) && (v == e_.size() || e_[i].tick < e_[v].tick)) v = i;
        if (v == e_.size()) return false;
        out.push_back(std::move(e_[v].img));
        e_.erase(e_.begin() + (long)v);
        return true;
    }
    // every idle image of dev (dev < 0: all GPUs); returns the bytes released
    uint64_t release_idle(int dev, Evicted &out) {
        uint64_t b = 0;
        for (size_t i = e_.size(); i-- > 0;)
            if ((dev < 0 || e_[i].dev == dev) && idle(e_[i])) {
                b += e_[i].bytes;
                out.push_back(std::move(e_[i].img));
                e_.erase(e_.begin() + (long)i);
            }
        return b;
    }

  private:
    std::vector<Entry> e_;
    uint64_t tick_ = 0;
};

}  // namespace fls
