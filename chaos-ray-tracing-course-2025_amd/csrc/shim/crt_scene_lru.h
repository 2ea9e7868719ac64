/*
 * crt_scene_lru.h — the shim's bounded cache of device scenes
 * (crt_render_image_hip.cpp).  A long-running host (the Python module, the
 * Blender add-on) builds a new crt::Scene per render; each cached entry owns
 * a device scene (full-resolution output, tile plans, ...), so the cache keeps
 * the `cap` most recently used entries and destroys the rest.  Entries are
 * found by content (a predicate), not by the Scene's address.
 */
#pragma once
#include <cstddef>
#include <list>
#include <memory>

namespace crt_shim {

template <class T>
class SceneLru {
  public:
    explicit SceneLru(size_t cap) : cap_(cap < 1 ? 1 : cap) {}

    /* the first entry satisfying pred, moved to the front; null if none */
    template <class Pred>
    T *find(Pred pred) {
        for (auto it = items_.begin(); it != items_.end(); ++it)
            if (pred(**it)) {
                items_.splice(items_.begin(), items_, it);
                return items_.front().get();
            }
        return nullptr;
    }

    /* insert at the front, destroying the least recently used beyond cap */
    T *insert(std::unique_ptr<T> v) {
        items_.push_front(std::move(v));
        while (items_.size() > cap_) items_.pop_back();
        return items_.front().get();
    }

    size_t size() const { return items_.size(); }
    void clear() { items_.clear(); }

  private:
    size_t cap_;
    std::list<std::unique_ptr<T>> items_;
};

}  // namespace crt_shim
