/*
 * ur3e_mjcf.cpp — the C ABI's MJCF and YAML entry points (include/ur3e_batch.h):
 *
 *   ur3e_model_from_mjcf          the reference's model file (assets/main.xml, loaded by
 *                                 gymnasium_env/envs/ur3e_env2.py:30-36 through MujocoEnv, and by
 *                                 init_mj.py:22-30 for the scripted drivers) -> ur3e_model_t
 *   ur3e_config_gains_from_yaml   the reference's gain files (ur3e_env2.py:66-68 and
 *                                 controller/move_l_mug.py:20-27: config_l_mug.yml; move_j.py:46-52:
 *                                 config_j.yml; move_l.py:92-99: config_l.yml) -> ur3e_config_t gains
 *   ur3e_batch_create_from_mjcf   both, then ur3e_batch_create
 *
 * The MJCF compiler (ur3e_amd/model/compiler.py: defaults classes, meshes, inertias, collision filter,
 * keyframes) and the YAML reader (ur3e_amd/gains.py) are the package's Python; a caller that is not
 * Python (C, Go over cgo, Java over JNI ...) reaches them here through an embedded interpreter: libpython
 * is loaded with dlopen on first use (no link-time dependency of the library), the package is found
 * beside this library (ur3e_amd/_lib/.. /..; UR3E_PYTHONPATH overrides), and the results come back as
 * files in a private temporary directory (ur3e_amd/model/image.py writes them: the raw ur3e_model_t, or
 * 36 doubles of gains).  In a Python process the running interpreter is used (the GIL is taken for the
 * call).  Nothing here touches the GPU.
 */
#include <dirent.h>
#include <dlfcn.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/ur3e_batch.h"
#include "gen_pyconfig.h"

__attribute__((visibility("hidden"))) int ur3e_internal_fail(int code, const char* msg);

namespace {

struct PyApi {
  int (*IsInitialized)(void) = nullptr;
  void (*InitializeEx)(int) = nullptr;
  int (*GILStateEnsure)(void) = nullptr; /* PyGILState_STATE is an enum */
  void (*GILStateRelease)(int) = nullptr;
  void* (*EvalSaveThread)(void) = nullptr;
  int (*RunSimpleStringFlags)(const char*, void*) = nullptr;
  bool ok = false;
};

int fail(int code, const std::string& msg) { return ur3e_internal_fail(code, msg.c_str()); }

bool load_python(PyApi& p, std::string& err) {
  static PyApi cached;
  if (cached.ok) {
    p = cached;
    return true;
  }
  /* a Python process: the interpreter's own symbols (a python binary with libpython linked in statically
     exports them); loading libpython beside it would start a second interpreter */
  void* h = RTLD_DEFAULT; /* (a null handle on glibc: `found` says whether it serves) */
  bool found = dlsym(RTLD_DEFAULT, "Py_IsInitialized") != nullptr;
  /* UR3E_LIBPYTHON, when set, is the only candidate; otherwise the libpython of the interpreter that built
     this library (gen_pyconfig.h, written by ur3e_amd/_build.py), then the same version's soname, then
     the stable-ABI soname */
  std::vector<std::string> names;
  if (const char* e = getenv("UR3E_LIBPYTHON")) {
    names.push_back(e);
  } else {
    names.push_back(UR3E_BUILD_LIBPYTHON);
    names.push_back(UR3E_BUILD_LIBPYTHON_SONAME);
    names.push_back("libpython3.so");
  }
  std::string last;
  for (size_t k = 0; !found && k < names.size(); k++) {
    if (names[k].empty()) continue;
    h = dlopen(names[k].c_str(), RTLD_NOW | RTLD_GLOBAL);
    found = h != nullptr;
    if (!found) {
      const char* de = dlerror(); /* read once: the call clears it */
      last = de ? de : "";
    }
  }
  if (!found) {
    err = "libpython not found (set UR3E_LIBPYTHON): " + last;
    return false;
  }
  PyApi q;
  q.IsInitialized = (int (*)(void))dlsym(h, "Py_IsInitialized");
  q.InitializeEx = (void (*)(int))dlsym(h, "Py_InitializeEx");
  q.GILStateEnsure = (int (*)(void))dlsym(h, "PyGILState_Ensure");
  q.GILStateRelease = (void (*)(int))dlsym(h, "PyGILState_Release");
  q.EvalSaveThread = (void* (*)(void))dlsym(h, "PyEval_SaveThread");
  q.RunSimpleStringFlags = (int (*)(const char*, void*))dlsym(h, "PyRun_SimpleStringFlags");
  if (!q.IsInitialized || !q.InitializeEx || !q.GILStateEnsure || !q.GILStateRelease || !q.EvalSaveThread ||
      !q.RunSimpleStringFlags) {
    err = "libpython lacks the embedding API";
    return false;
  }
  q.ok = true;
  cached = q;
  p = q;
  return true;
}

/* a Python str expression for s: a bytes literal (every byte >= 128 or < 32 escaped) decoded with the
   filesystem encoding, so that a path's non-ASCII bytes arrive as the same path (a str literal would read
   each escaped byte as a code point) */
std::string pyquote(const std::string& s) {
  std::string o = "__import__('os').fsdecode(b'";
  for (unsigned char ch : s) {
    if (ch == '\\' || ch == '\'') {
      o += '\\';
      o += (char)ch;
    } else if (ch < 32 || ch >= 127) {
      char buf[8];
      snprintf(buf, sizeof buf, "\\x%02x", ch);
      o += buf;
    } else {
      o += (char)ch;
    }
  }
  return o + "')";
}

/* the directory holding the ur3e_amd package: two levels above this library (ur3e_amd/_lib/x.so) */
std::string package_root() {
  if (const char* e = getenv("UR3E_PYTHONPATH")) return e;
  Dl_info info;
  if (!dladdr((void*)&package_root, &info) || !info.dli_fname) return ".";
  std::string p = info.dli_fname;
  for (int k = 0; k < 3; k++) {
    const size_t s = p.find_last_of('/');
    if (s == std::string::npos) return ".";
    p = p.substr(0, s);
  }
  return p.empty() ? "/" : p;
}

struct TmpDir {
  std::string path;
  TmpDir() {
    const char* t = getenv("TMPDIR");
    std::string tmpl = std::string(t && *t ? t : "/tmp") + "/ur3e_mjcf_XXXXXX";
    std::vector<char> b(tmpl.begin(), tmpl.end());
    b.push_back(0);
    if (mkdtemp(b.data())) path = b.data();
  }
  ~TmpDir() {
    if (path.empty()) return;
    if (DIR* d = opendir(path.c_str())) {
      while (dirent* e = readdir(d)) {
        if (!strcmp(e->d_name, ".") || !strcmp(e->d_name, "..")) continue;
        unlink((path + "/" + e->d_name).c_str());
      }
      closedir(d);
    }
    rmdir(path.c_str());
  }
};

bool read_file(const std::string& path, std::vector<char>& out) {
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) return false;
  out.clear();
  char buf[65536];
  size_t k;
  while ((k = fread(buf, 1, sizeof buf, f)) > 0) out.insert(out.end(), buf, buf + k);
  fclose(f);
  return true;
}

/* run `body` (Python statements, indented by 4) with the package importable; an exception's repr goes
   to <dir>/err, which is returned as the error message */
int run_python(const std::string& dir, const std::string& body, std::string& err) {
  PyApi p;
  if (!load_python(p, err)) return UR3E_EINVAL;
  if (!p.IsInitialized()) {
    p.InitializeEx(0);
    p.EvalSaveThread(); /* release the GIL this thread holds after initialisation */
  }
  const std::string code = "import sys\n"
                           "_r = " + pyquote(package_root()) + "\n"
                           "if _r not in sys.path:\n    sys.path.insert(0, _r)\n"
                           "try:\n" + body +
                           "except BaseException as _e:\n"
                           "    import traceback\n"
                           "    open(" + pyquote(dir + "/err") + ", 'w').write(''.join(traceback.format_exception_only(type(_e), _e)))\n";
  /* in a namespace of its own: nothing lands in the host interpreter's __main__ */
  const std::string src = "exec(" + pyquote(code) + ", {})\n";
  const int g = p.GILStateEnsure();
  const int rc = p.RunSimpleStringFlags(src.c_str(), nullptr);
  p.GILStateRelease(g);
  std::vector<char> e;
  if (read_file(dir + "/err", e)) {
    err.assign(e.begin(), e.end());
    while (!err.empty() && (err.back() == '\n' || err.back() == ' ')) err.pop_back();
    return UR3E_EINVAL;
  }
  if (rc != 0) {
    err = "embedded Python failed";
    return UR3E_EINVAL;
  }
  return UR3E_OK;
}

}  // namespace

extern "C" int ur3e_model_from_mjcf(const char* mjcf_path, const char* meshes, ur3e_model_t* out) {
  if (!mjcf_path || !out) return fail(UR3E_EINVAL, "null argument");
  const std::string mode = meshes && *meshes ? meshes : "auto";
  if (mode != "auto" && mode != "mesh" && mode != "surrogate") return fail(UR3E_EINVAL, "meshes: auto, mesh or surrogate");
  struct stat st;
  if (stat(mjcf_path, &st) != 0) return fail(UR3E_EINVAL, std::string("no such MJCF file: ") + mjcf_path);
  TmpDir t;
  if (t.path.empty()) return fail(UR3E_EINVAL, "cannot create a temporary directory");
  const std::string img = t.path + "/model.bin";
  std::string err;
  const int rc = run_python(t.path,
                            "    from ur3e_amd.model import image as _img\n"
                            "    _img.write_model_image(" + pyquote(mjcf_path) + ", " + pyquote(img) + ", " +
                                pyquote(mode) + ")\n",
                            err);
  if (rc != UR3E_OK) return fail(rc, "ur3e_model_from_mjcf(" + std::string(mjcf_path) + "): " + err);
  std::vector<char> raw;
  if (!read_file(img, raw)) return fail(UR3E_EINVAL, "model image missing");
  if (raw.size() != sizeof(ur3e_model_t))
    return fail(UR3E_EINVAL, "model image is " + std::to_string(raw.size()) + " bytes, ur3e_model_t " +
                                 std::to_string(sizeof(ur3e_model_t)) + " (package and library out of step)");
  memcpy(out, raw.data(), sizeof(ur3e_model_t));
  return UR3E_OK;
}

extern "C" int ur3e_config_gains_from_yaml(const char* config_yaml_path, ur3e_config_t* cfg) {
  if (!cfg) return fail(UR3E_EINVAL, "null config");
  TmpDir t;
  if (t.path.empty()) return fail(UR3E_EINVAL, "cannot create a temporary directory");
  const std::string out = t.path + "/gains.bin";
  std::string err;
  const std::string yml = config_yaml_path && *config_yaml_path ? pyquote(config_yaml_path) : "None";
  const int rc = run_python(t.path,
                            "    from ur3e_amd.model import image as _img\n"
                            "    _img.write_gains(" + yml + ", " + std::to_string(cfg->task) + ", " + pyquote(out) +
                                ")\n",
                            err);
  if (rc != UR3E_OK) return fail(rc, "ur3e_config_gains_from_yaml: " + err);
  std::vector<char> raw;
  if (!read_file(out, raw) || raw.size() != 36 * sizeof(double)) return fail(UR3E_EINVAL, "gains file malformed");
  const double* g = (const double*)raw.data();
  memcpy(cfg->task_gains, g, 12 * sizeof(double));
  memcpy(cfg->joint_gains, g + 12, 12 * sizeof(double));
  memcpy(cfg->rot_joint_gains, g + 24, 12 * sizeof(double));
  return UR3E_OK;
}

extern "C" int ur3e_batch_create_from_mjcf(const char* mjcf_path, const char* config_yaml_path, const ur3e_config_t* cfg,
                                           int n_envs, int device, ur3e_batch_t** out) {
  if (!mjcf_path || !cfg || !out) return fail(UR3E_EINVAL, "null argument");
  ur3e_model_t* m = (ur3e_model_t*)malloc(sizeof(ur3e_model_t));
  if (!m) return fail(UR3E_EINVAL, "out of host memory");
  int rc = ur3e_model_from_mjcf(mjcf_path, "auto", m);
  if (rc == UR3E_OK) {
    ur3e_config_t c = *cfg;
    rc = ur3e_config_gains_from_yaml(config_yaml_path, &c);
    if (rc == UR3E_OK) rc = ur3e_batch_create(m, &c, n_envs, device, out);
  }
  free(m);
  return rc;
}
