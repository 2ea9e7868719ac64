/*
 * _crt — CPython module, drop-in for src/python/py_crt_module.cpp (the module
 * the Blender add-on imports, bl_crt_engine.py:13-30).
 *
 *   _crt.RendererSettings((max_ray_depth, diffuse_reflection_ray_count, shadow_bias,
 *                          reflection_bias, diffuse_reflection_bias, refraction_bias))
 *   _crt.render_scene_from_dict(dict, asset_root: str, settings) -> list[(r, g, b, 1.0)]
 *   _crt.DEFAULT_SCENE_BUCKET_SIZE, DEFAULT_MAX_RAY_DEPTH, ... (py_crt_module.cpp:142-157)
 *
 * Same argument parsing ("O!UO"), same json.dumps(ensure_ascii=True) hand-off
 * to the loader, same errors (ValueError "Invalid CRT Scene dict", TypeError
 * "Expected a RendererSettings instance"), same bottom-up row order of the
 * returned RGBA list (:102-116).  Differences: the render runs on the GPU
 * through lib/libcrt_hip.so with the GIL released, a HIP failure raises
 * RuntimeError, and the json.dumps argument tuple is not leaked (:73).
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <structmember.h>

#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../../include/crt_hip.h"

/* the device scene of the last rendered dict (render_scene_from_dict), keyed
 * by everything but the camera (geometry, materials, textures with their
 * texels, lights, background, flags): a dict that differs only in its camera
 * moves the kept scene's camera instead of uploading the scene again */
static std::mutex g_scene_mu;
static crt_hip_scene *g_scene = nullptr;
static std::string g_scene_key;
static long long g_creates = 0, g_camera_moves = 0, g_reuses = 0;

template <class T>
static void key_put(std::string &k, const T *p, size_t n) {
    const uint64_t nb = (uint64_t)(n * sizeof(T));
    k.append(reinterpret_cast<const char *>(&nb), sizeof nb);
    if (p && n) k.append(reinterpret_cast<const char *>(p), n * sizeof(T));
}

/* The scene without its camera, as bytes. */
static std::string scene_key(const crt_scene_desc *d, const char *root, size_t rn) {
    std::string k(root, rn);
    k.push_back('\0');
    key_put(k, &d->background_color, 1);
    const int32_t flags[4] = {d->bucket_size, d->gi_on, d->reflections_on, d->refractions_on};
    key_put(k, flags, 4);
    key_put(k, &d->mesh_count, 1);
    for (int32_t i = 0; i < d->mesh_count; ++i) {
        const crt_mesh_desc &m = d->meshes[i];
        key_put(k, m.positions, (size_t)m.vertex_count * 3);
        key_put(k, m.uvs, m.uvs ? (size_t)m.vertex_count * 3 : 0);
        key_put(k, m.indices, (size_t)m.index_count);
        key_put(k, &m.material_index, 1);
    }
    key_put(k, d->materials, (size_t)d->material_count);
    key_put(k, d->lights, (size_t)d->light_count);
    key_put(k, &d->texture_count, 1);
    for (int32_t i = 0; i < d->texture_count; ++i) {
        const crt_texture_desc &t = d->textures[i];
        const float f[7] = {t.color0.x, t.color0.y, t.color0.z, t.color1.x, t.color1.y, t.color1.z, t.scalar};
        const int32_t ti[3] = {t.type, t.bitmap_width, t.bitmap_height};
        key_put(k, ti, 3);
        key_put(k, f, 7);
        /* bitmap textures are read from disk by every parse (as the reference
         * reloads them every call): their decoded texels are part of the key,
         * so an edited texture file never reuses the kept device scene */
        if (t.type == CRT_TEXTURE_BITMAP && t.bitmap_rgb)
            key_put(k, t.bitmap_rgb, (size_t)t.bitmap_width * t.bitmap_height * 3);
    }
    return k;
}

static bool same_camera(const crt_hip_scene *sc, const crt_camera_desc &c) {
    crt_camera_desc cur;
    float fov = 0.f;
    if (crt_hip_scene_camera(sc, &cur, &fov) != CRT_OK) return false;
    const float want = c.fov_degrees * 3.14159265358979323846f / 180.0f;   /* crt_camera.h:20 */
    return cur.location.x == c.location.x && cur.location.y == c.location.y && cur.location.z == c.location.z &&
           std::memcmp(cur.rotation, c.rotation, sizeof cur.rotation) == 0 && cur.width == c.width &&
           cur.height == c.height && fov == want;
}

static PyStructSequence_Field settings_fields[] = {
    {(char *)"max_ray_depth", (char *)"Maximum recursion depth for rays"},
    {(char *)"diffuse_reflection_ray_count", (char *)"Number of rays for diffuse reflections"},
    {(char *)"shadow_bias", (char *)"Epsilon used for shadow acne avoidance"},
    {(char *)"reflection_bias", (char *)"Epsilon used for reflection acne avoidance"},
    {(char *)"diffuse_reflection_bias", (char *)"Epsilon used for diffuse reflection acne avoidance"},
    {(char *)"refraction_bias", (char *)"Epsilon used for refraction acne avoidance"},
    {nullptr, nullptr}};

static PyStructSequence_Desc settings_desc = {(char *)"_crt.RendererSettings",
                                              (char *)"Renderer settings used by crt_core", settings_fields, 6};

static PyTypeObject *SettingsType = nullptr;

static bool get_settings(PyObject *obj, crt_renderer_settings &out) {
    if (!PyObject_TypeCheck(obj, SettingsType)) {
        PyErr_SetString(PyExc_TypeError, "Expected a RendererSettings instance");
        return false;
    }
    out.max_ray_depth = (uint32_t)PyLong_AsUnsignedLong(PyStructSequence_GET_ITEM(obj, 0));
    out.diffuse_reflection_ray_count = (uint32_t)PyLong_AsUnsignedLong(PyStructSequence_GET_ITEM(obj, 1));
    out.shadow_bias = (float)PyFloat_AsDouble(PyStructSequence_GET_ITEM(obj, 2));
    out.reflection_bias = (float)PyFloat_AsDouble(PyStructSequence_GET_ITEM(obj, 3));
    out.diffuse_reflection_bias = (float)PyFloat_AsDouble(PyStructSequence_GET_ITEM(obj, 4));
    out.refraction_bias = (float)PyFloat_AsDouble(PyStructSequence_GET_ITEM(obj, 5));
    return !PyErr_Occurred();
}

static PyObject *render_scene_from_dict(PyObject *, PyObject *args) {
    PyObject *dict_obj, *asset_root, *settings_obj;
    if (!PyArg_ParseTuple(args, "O!UO", &PyDict_Type, &dict_obj, &asset_root, &settings_obj)) return nullptr;

    PyObject *json_mod = PyImport_ImportModule("json");
    if (!json_mod) return nullptr;
    PyObject *dumps = PyObject_GetAttrString(json_mod, "dumps");
    Py_DECREF(json_mod);
    if (!dumps) return nullptr;
    PyObject *kwargs = Py_BuildValue("{sO}", "ensure_ascii", Py_True);
    PyObject *pargs = PyTuple_Pack(1, dict_obj);
    PyObject *text = (kwargs && pargs) ? PyObject_Call(dumps, pargs, kwargs) : nullptr;
    Py_XDECREF(kwargs);
    Py_XDECREF(pargs);
    Py_DECREF(dumps);
    if (!text) return nullptr;

    Py_ssize_t n = 0;
    const char *utf8 = PyUnicode_AsUTF8AndSize(text, &n);
    Py_ssize_t rn = 0;
    const char *root = PyUnicode_AsUTF8AndSize(asset_root, &rn);
    if (!utf8 || !root) {
        Py_DECREF(text);
        return nullptr;
    }
    crt_scene_file *sf = nullptr;
    const int prc = crt_scene_file_parse(utf8, (size_t)n, root, &sf);
    Py_DECREF(text);
    if (prc != CRT_OK) {
        PyErr_SetString(PyExc_ValueError, "Invalid CRT Scene dict");
        return nullptr;
    }
    crt_renderer_settings st;
    if (!get_settings(settings_obj, st)) {
        crt_scene_file_destroy(sf);
        return nullptr;
    }
    const crt_scene_desc *desc = crt_scene_file_desc(sf);
    const int W = desc->camera.width, H = desc->camera.height;
    std::vector<float> img((size_t)W * H * 3);
    int rc;
    std::string err;
    Py_BEGIN_ALLOW_THREADS
    {
        /* the device scene of the last dict is kept (a Blender session
         * re-renders the same scene with other settings, or with the camera
         * moved from frame to frame): the same scene without its camera and
         * the same asset root -> no new upload, the camera moved in place, and
         * the measured tile plan stays */
        const std::string key = scene_key(desc, root, (size_t)rn);
        std::lock_guard<std::mutex> lock(g_scene_mu);
        if (!g_scene || g_scene_key != key) {
            crt_hip_scene_destroy(g_scene);
            g_scene = nullptr;
            g_scene_key.clear();
            rc = crt_hip_scene_create_auto(desc, &st, CRT_SCENE_TREE_AUTO, &g_scene);   /* GPUs the frame pays for */
            if (rc == CRT_OK) {
                g_scene_key = key;
                ++g_creates;
            }
        } else if (!same_camera(g_scene, desc->camera)) {
            rc = crt_hip_scene_set_camera(g_scene, &desc->camera);
            ++g_camera_moves;
        } else {
            rc = CRT_OK;
            ++g_reuses;
        }
        if (rc == CRT_OK) rc = crt_hip_render(g_scene, &st, img.data(), nullptr);
        if (rc != CRT_OK) {
            err = crt_hip_last_error();
            crt_hip_scene_destroy(g_scene);
            g_scene = nullptr;
            g_scene_key.clear();
        }
    }
    Py_END_ALLOW_THREADS
    crt_scene_file_destroy(sf);
    if (rc != CRT_OK) {
        PyErr_SetString(PyExc_RuntimeError, err.c_str());
        return nullptr;
    }
    PyObject *list = PyList_New((Py_ssize_t)W * H);
    if (!list) return nullptr;
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            const float *c = &img[3 * ((size_t)y * W + x)];
            PyObject *t = Py_BuildValue("ffff", c[0], c[1], c[2], 1.0f);
            if (!t) {
                Py_DECREF(list);
                return nullptr;
            }
            PyList_SET_ITEM(list, (Py_ssize_t)(H - y - 1) * W + x, t);
        }
    return list;
}

/* Diagnostics (not in the reference module): how render_scene_from_dict
 * treated the calls so far — new device scenes, camera moves of the kept one,
 * reuses as they were. */
static PyObject *device_scene_stats(PyObject *, PyObject *) {
    std::lock_guard<std::mutex> lock(g_scene_mu);
    return Py_BuildValue("{sLsLsL}", "creates", g_creates, "camera_moves", g_camera_moves, "reuses", g_reuses);
}

static PyMethodDef methods[] = {
    {"render_scene_from_dict", (PyCFunction)render_scene_from_dict, METH_VARARGS,
     "render_scene_from_dict(scene_dict, asset_root, settings) -> list of (r, g, b, a), bottom row first"},
    {"_device_scene_stats", (PyCFunction)device_scene_stats, METH_NOARGS,
     "diagnostics: {creates, camera_moves, reuses} of render_scene_from_dict's kept device scene"},
    {nullptr, nullptr, 0, nullptr}};

static PyModuleDef module_def = {PyModuleDef_HEAD_INIT, "_crt", nullptr, -1, methods};

PyMODINIT_FUNC PyInit__crt(void) {
    PyObject *m = PyModule_Create(&module_def);
    if (!m) return nullptr;
    crt_renderer_settings d;
    crt_renderer_settings_default(&d);
    if (PyModule_AddIntConstant(m, "DEFAULT_SCENE_BUCKET_SIZE", 24) < 0 ||
        PyModule_AddIntConstant(m, "DEFAULT_MAX_RAY_DEPTH", (long)d.max_ray_depth) < 0 ||
        PyModule_AddIntConstant(m, "DEFAULT_DIFFUSE_REFLECTION_RAY_COUNT", (long)d.diffuse_reflection_ray_count) < 0 ||
        PyModule_AddObject(m, "DEFAULT_SHADOW_BIAS", PyFloat_FromDouble(d.shadow_bias)) < 0 ||
        PyModule_AddObject(m, "DEFAULT_REFLECTION_BIAS", PyFloat_FromDouble(d.reflection_bias)) < 0 ||
        PyModule_AddObject(m, "DEFAULT_DIFFUSE_REFLECTION_BIAS", PyFloat_FromDouble(d.diffuse_reflection_bias)) < 0 ||
        PyModule_AddObject(m, "DEFAULT_REFRACTION_BIAS", PyFloat_FromDouble(d.refraction_bias)) < 0) {
        Py_DECREF(m);
        return nullptr;
    }
    SettingsType = PyStructSequence_NewType(&settings_desc);
    if (!SettingsType) {
        Py_DECREF(m);
        return nullptr;
    }
    Py_INCREF(SettingsType);
    if (PyModule_AddObject(m, "RendererSettings", (PyObject *)SettingsType) < 0) {
        Py_DECREF(SettingsType);
        Py_DECREF(m);
        return nullptr;
    }
    return m;
}
