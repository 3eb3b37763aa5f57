// arena.h -- device address-space allocator of the HIP driver.
//
// Plays the role of runtime/common/malloc.h:22-542 (MemoryAllocator: page
// 4 KB / block 64 B, base USER_BASE_ADDR) but over one contiguous HBM arena:
// a device address is an offset into the arena, so it stays small enough for
// the 32-bit `addr / 64` DCRs the apps write (draw3d/main.cpp:216-230), and a
// kernel turns it into a pointer with one add (vx_ptr<T>() in vx_spawn.h).
// First-fit over an address-ordered free list with neighbour coalescing.
#pragma once

#include <cstdint>
#include <map>

class ArenaAllocator {
 public:
  ArenaAllocator(uint64_t base, uint64_t size, uint64_t align)
      : base_(base), size_(size), align_(align) {
    if (size > 0) free_[base] = size;
  }

  int allocate(uint64_t size, uint64_t* addr) {
    if (size == 0 || addr == nullptr) return -1;
    const uint64_t asize = align_up(size);
    for (auto it = free_.begin(); it != free_.end(); ++it) {
      if (it->second < asize) continue;
      const uint64_t a = it->first, fsize = it->second;
      free_.erase(it);
      if (fsize > asize) free_[a + asize] = fsize - asize;
      used_[a] = asize;
      *addr = a;
      return 0;
    }
    return -1;  // out of device memory
  }

  int reserve(uint64_t addr, uint64_t size) {
    if (size == 0 || (addr % align_) != 0) return -1;
    const uint64_t asize = align_up(size);
    auto it = free_.upper_bound(addr);
    if (it == free_.begin()) return -1;
    --it;
    const uint64_t fa = it->first, fs = it->second;
    if (addr < fa || addr + asize > fa + fs) return -1;  // not entirely free
    free_.erase(it);
    if (addr > fa) free_[fa] = addr - fa;
    if (addr + asize < fa + fs) free_[addr + asize] = fa + fs - (addr + asize);
    used_[addr] = asize;
    return 0;
  }

  int release(uint64_t addr) {
    auto it = used_.find(addr);
    if (it == used_.end()) return -1;
    uint64_t a = addr, s = it->second;
    used_.erase(it);
    auto nx = free_.lower_bound(a);
    if (nx != free_.end() && a + s == nx->first) {  // merge with next
      s += nx->second;
      nx = free_.erase(nx);
    }
    if (nx != free_.begin()) {                       // merge with previous
      auto pv = std::prev(nx);
      if (pv->first + pv->second == a) {
        pv->second += s;
        return 0;
      }
    }
    free_[a] = s;
    return 0;
  }

  // size of the allocation that contains `addr` (0 if none); start in *start
  uint64_t find(uint64_t addr, uint64_t* start) const {
    auto it = used_.upper_bound(addr);
    if (it == used_.begin()) return 0;
    --it;
    if (addr >= it->first + it->second) return 0;
    if (start) *start = it->first;
    return it->second;
  }

  uint64_t free_bytes() const {
    uint64_t s = 0;
    for (auto& kv : free_) s += kv.second;
    return s;
  }
  uint64_t used_bytes() const {
    uint64_t s = 0;
    for (auto& kv : used_) s += kv.second;
    return s;
  }
  uint64_t base() const { return base_; }
  uint64_t end() const { return base_ + size_; }

 private:
  uint64_t align_up(uint64_t v) const { return (v + align_ - 1) / align_ * align_; }
  uint64_t base_, size_, align_;
  std::map<uint64_t, uint64_t> free_;
  std::map<uint64_t, uint64_t> used_;
};
