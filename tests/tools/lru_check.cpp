/* TEST TOOL (CPU only): the shim's scene cache (csrc/shim/crt_scene_lru.h)
 * stays bounded and destroys what it evicts.  Prints "ok" or the failure. */
#include <cstdio>
#include <memory>

#include "../../chaos-ray-tracing-course-2025_amd/csrc/shim/crt_scene_lru.h"

static int g_live = 0;
struct Entry {
    int key;
    explicit Entry(int k) : key(k) { ++g_live; }
    ~Entry() { --g_live; }
};

int main() {
    crt_shim::SceneLru<Entry> c(2);
    for (int k = 0; k < 50; ++k) {   /* 50 distinct scenes in a row */
        if (c.find([&](const Entry &e) { return e.key == k; })) { std::puts("found a scene never inserted"); return 1; }
        c.insert(std::unique_ptr<Entry>(new Entry(k)));
        if (c.size() > 2 || g_live > 2) { std::printf("cache grew: %zu entries, %d live\n", c.size(), g_live); return 1; }
    }
    /* the two most recent are kept, found by content, and a hit refreshes */
    if (!c.find([](const Entry &e) { return e.key == 48; })) { std::puts("lost key 48"); return 1; }
    c.insert(std::unique_ptr<Entry>(new Entry(99)));   /* evicts 49, the least recently used */
    if (!c.find([](const Entry &e) { return e.key == 48; }) || c.find([](const Entry &e) { return e.key == 49; })) {
        std::puts("wrong eviction order");
        return 1;
    }
    c.clear();
    if (g_live != 0) { std::puts("entries leaked"); return 1; }
    std::puts("ok");
    return 0;
}
