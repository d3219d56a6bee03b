// Launch timeline bookkeeping (host side of TLScope, csrc/kernels/common.h).
// One device buffer of u64 stamps is handed out slot by slot to kernel launches while a
// timeline is active; the (name, offset, blocks) records let benchmarks/timeline.py map the
// stamps back to launches. A captured hipGraph keeps the slots it was captured with.
#include <string>
#include <vector>

#include "../kernels/launchers.h"

namespace vgate {
namespace {
struct Entry {
  std::string name;
  int64_t off;
  int nblk;
};
unsigned long long* g_base = nullptr;
int64_t g_cap = 0, g_used = 0;
std::vector<Entry> g_entries;
}  // namespace

unsigned long long* tl_take(const char* name, int nblocks) {
  if (g_base == nullptr || nblocks <= 0 || g_used + 2 * (int64_t)nblocks > g_cap) return nullptr;
  unsigned long long* p = g_base + g_used;
  g_entries.push_back({name, g_used, nblocks});
  g_used += 2 * (int64_t)nblocks;
  return p;
}

void tl_start(unsigned long long* base, int64_t capacity) {
  g_base = base;
  g_cap = capacity;
  g_used = 0;
  g_entries.clear();
}

int64_t tl_stop() {
  g_base = nullptr;
  return g_used;
}

int tl_count() { return (int)g_entries.size(); }
const char* tl_name(int i) { return g_entries.at(i).name.c_str(); }
int64_t tl_offset(int i) { return g_entries.at(i).off; }
int tl_blocks(int i) { return g_entries.at(i).nblk; }

}  // namespace vgate
