#include "file_mgr.h"

#include <sys/stat.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <cstdlib>
#include <filesystem>
#include <sstream>
#include <system_error>

namespace pbx {

namespace fs = std::filesystem;

namespace {

std::string quote(const std::string& s) {
  std::string o = "'";
  for (char c : s) {
    if (c == '\'')
      o += "'\\''";
    else
      o += c;
  }
  return o + "'";
}

bool ends_with(const std::string& s, const std::string& suf) {
  return s.size() >= suf.size() && s.compare(s.size() - suf.size(), suf.size(), suf) == 0;
}

std::string strip_file_scheme(const std::string& p) { return p.rfind("file:", 0) == 0 ? p.substr(5) : p; }

int64_t tree_bytes(const fs::path& p) {
  std::error_code ec;
  if (fs::is_regular_file(p, ec)) return (int64_t)fs::file_size(p, ec);
  int64_t tot = 0;
  for (auto it = fs::recursive_directory_iterator(p, ec); !ec && it != fs::recursive_directory_iterator();
       it.increment(ec))
    if (it->is_regular_file(ec)) tot += (int64_t)it->file_size(ec);
  return tot;
}

// `hadoop fs -ls` lines: "perm repl user group size date time path"
bool parse_ls_line(const std::string& line, std::string* path, int64_t* size) {
  std::istringstream is(line);
  std::vector<std::string> tok;
  std::string t;
  while (is >> t) tok.push_back(t);
  if (tok.size() < 8 || tok[0].empty() || (tok[0][0] != '-' && tok[0][0] != 'd')) return false;
  *path = tok.back();
  *size = std::atoll(tok[4].c_str());
  return true;
}

}  // namespace

bool FileMgr::init(const std::string& fs_name, const std::string& fs_ugi, const std::string& conf_path,
                   const std::string& hadoop_bin) {
  std::lock_guard<std::mutex> g(mu_);
  fs_name_ = fs_name;
  fs_ugi_ = fs_ugi;
  conf_path_ = conf_path;
  if (!hadoop_bin.empty()) {
    hadoop_bin_ = hadoop_bin;
  } else if (const char* hh = std::getenv("HADOOP_HOME")) {
    hadoop_bin_ = std::string(hh) + "/bin/hadoop";
  } else {
    hadoop_bin_ = "hadoop";
  }
  inited_ = true;
  return true;
}

void FileMgr::destroy() {
  std::lock_guard<std::mutex> g(mu_);
  inited_ = false;
}

bool FileMgr::is_remote(const std::string& path) {
  return path.rfind("hdfs://", 0) == 0 || path.rfind("afs://", 0) == 0 || path.rfind("hdfs:", 0) == 0 ||
         path.rfind("afs:", 0) == 0;
}

std::string FileMgr::remote_prefix() const {
  std::string p = quote(hadoop_bin_) + " fs";
  if (!conf_path_.empty()) p = quote(hadoop_bin_) + " --config " + quote(conf_path_) + " fs";
  if (!fs_name_.empty()) p += " -D fs.default.name=" + quote(fs_name_);
  if (!fs_ugi_.empty()) p += " -D hadoop.job.ugi=" + quote(fs_ugi_);
  return p + " ";
}

int FileMgr::run(const std::string& cmd, std::string* out) const {
  {
    std::lock_guard<std::mutex> g(mu_);
    last_cmd_ = cmd;
  }
  FILE* p = popen((cmd + " 2>/dev/null").c_str(), "r");
  if (!p) return -1;
  char buf[4096];
  size_t n;
  while ((n = fread(buf, 1, sizeof(buf), p)) > 0)
    if (out) out->append(buf, n);
  const int st = pclose(p);
  return WIFEXITED(st) ? WEXITSTATUS(st) : -1;
}

std::string FileMgr::last_command() const {
  std::lock_guard<std::mutex> g(mu_);
  return last_cmd_;
}

FILE* FileMgr::open_read(const std::string& path, const std::string& pipe_command, bool* is_pipe) const {
  const bool remote = is_remote(path);
  const bool gz = ends_with(path, ".gz");
  const bool convert = !pipe_command.empty() && pipe_command != "cat";
  if (!remote && !gz && !convert) {
    *is_pipe = false;
    return fopen(strip_file_scheme(path).c_str(), "r");
  }
  std::string cmd;
  if (remote) {
    cmd = remote_prefix() + (gz ? "-text " : "-cat ") + quote(path);  // -text decompresses
  } else {
    cmd = std::string(gz ? "zcat " : "cat ") + quote(strip_file_scheme(path));
  }
  if (convert) cmd += " | " + pipe_command;
  *is_pipe = true;
  {
    std::lock_guard<std::mutex> g(mu_);
    last_cmd_ = cmd;
  }
  return popen(cmd.c_str(), "r");
}

FILE* FileMgr::open_write(const std::string& path, bool* is_pipe) const {
  const bool gz = ends_with(path, ".gz");
  if (!is_remote(path) && !gz) {
    *is_pipe = false;
    const std::string lp = strip_file_scheme(path);
    std::error_code ec;
    fs::create_directories(fs::path(lp).parent_path(), ec);
    return fopen(lp.c_str(), "w");
  }
  std::string cmd;
  if (is_remote(path)) {
    cmd = (gz ? std::string("gzip -c | ") : std::string()) + remote_prefix() + "-put -f - " + quote(path);
  } else {
    cmd = "gzip -c > " + quote(strip_file_scheme(path));
  }
  *is_pipe = true;
  return popen(cmd.c_str(), "w");
}

void FileMgr::close(FILE* f, bool is_pipe) {
  if (!f) return;
  if (is_pipe)
    pclose(f);
  else
    fclose(f);
}

std::vector<std::pair<std::string, int64_t>> FileMgr::list_info(const std::string& path) const {
  std::vector<std::pair<std::string, int64_t>> out;
  if (is_remote(path)) {
    std::string o;
    if (run(remote_prefix() + "-ls " + quote(path), &o) != 0) return out;
    std::istringstream is(o);
    std::string line, p;
    int64_t sz;
    while (std::getline(is, line))
      if (parse_ls_line(line, &p, &sz)) out.emplace_back(p, sz);
  } else {
    std::error_code ec;
    const fs::path lp(strip_file_scheme(path));
    if (fs::is_directory(lp, ec)) {
      for (auto& e : fs::directory_iterator(lp, ec))
        out.emplace_back(e.path().string(), e.is_regular_file(ec) ? (int64_t)e.file_size(ec) : 0);
    } else if (fs::exists(lp, ec)) {
      out.emplace_back(lp.string(), (int64_t)fs::file_size(lp, ec));
    }
  }
  std::sort(out.begin(), out.end());
  return out;
}

std::vector<std::string> FileMgr::list_dir(const std::string& path) const {
  std::vector<std::string> out;
  for (auto& e : list_info(path)) out.push_back(e.first);
  return out;
}

bool FileMgr::makedir(const std::string& path) const {
  if (is_remote(path)) return run(remote_prefix() + "-mkdir -p " + quote(path), nullptr) == 0;
  std::error_code ec;
  fs::create_directories(strip_file_scheme(path), ec);
  return !ec;
}

bool FileMgr::exists(const std::string& path) const {
  if (is_remote(path)) return run(remote_prefix() + "-test -e " + quote(path), nullptr) == 0;
  std::error_code ec;
  return fs::exists(strip_file_scheme(path), ec);
}

bool FileMgr::download(const std::string& remote, const std::string& local) const {
  std::error_code ec;
  fs::create_directories(fs::path(local).parent_path(), ec);
  if (is_remote(remote)) return run(remote_prefix() + "-get " + quote(remote) + " " + quote(local), nullptr) == 0;
  fs::copy(strip_file_scheme(remote), local,
           fs::copy_options::recursive | fs::copy_options::overwrite_existing, ec);
  return !ec;
}

bool FileMgr::upload(const std::string& local, const std::string& remote) const {
  if (is_remote(remote)) return run(remote_prefix() + "-put -f " + quote(local) + " " + quote(remote), nullptr) == 0;
  return download(local, strip_file_scheme(remote));
}

bool FileMgr::remove(const std::string& path) const {
  if (is_remote(path)) return run(remote_prefix() + "-rm -r -f " + quote(path), nullptr) == 0;
  std::error_code ec;
  fs::remove_all(strip_file_scheme(path), ec);
  return !ec;
}

int64_t FileMgr::file_size(const std::string& path) const {
  if (is_remote(path)) {
    auto li = list_info(path);
    return li.size() == 1 ? li[0].second : -1;
  }
  std::error_code ec;
  const auto s = fs::file_size(strip_file_scheme(path), ec);
  return ec ? -1 : (int64_t)s;
}

std::vector<std::pair<std::string, int64_t>> FileMgr::dus(const std::string& path) const {
  std::vector<std::pair<std::string, int64_t>> out;
  if (is_remote(path)) {
    // `-du` lines: "<size> [<size with replication>] <path>"
    std::string o;
    if (run(remote_prefix() + "-du " + quote(path), &o) != 0) return out;
    std::istringstream is(o);
    std::string line;
    while (std::getline(is, line)) {
      std::istringstream ls(line);
      std::vector<std::string> tok;
      std::string t;
      while (ls >> t) tok.push_back(t);
      if (tok.size() >= 2) out.emplace_back(tok.back(), std::atoll(tok[0].c_str()));
    }
  } else {
    std::error_code ec;
    const fs::path lp(strip_file_scheme(path));
    if (fs::is_directory(lp, ec)) {
      for (auto& e : fs::directory_iterator(lp, ec)) out.emplace_back(e.path().string(), tree_bytes(e.path()));
    } else if (fs::exists(lp, ec)) {
      out.emplace_back(lp.string(), tree_bytes(lp));
    }
  }
  std::sort(out.begin(), out.end());
  return out;
}

bool FileMgr::truncate(const std::string& path, int64_t len) const {
  if (is_remote(path)) return run(remote_prefix() + "-truncate -w " + std::to_string(len) + " " + quote(path), nullptr) == 0;
  return ::truncate(strip_file_scheme(path).c_str(), (off_t)len) == 0;
}

bool FileMgr::touch(const std::string& path) const {
  if (is_remote(path)) return run(remote_prefix() + "-touchz " + quote(path), nullptr) == 0;
  const std::string lp = strip_file_scheme(path);
  std::error_code ec;
  fs::create_directories(fs::path(lp).parent_path(), ec);
  FILE* f = fopen(lp.c_str(), "a");
  if (!f) return false;
  fclose(f);
  return true;
}

bool FileMgr::rename(const std::string& src, const std::string& dst) const {
  if (is_remote(src) || is_remote(dst))
    return run(remote_prefix() + "-mv " + quote(src) + " " + quote(dst), nullptr) == 0;
  std::error_code ec;
  fs::rename(strip_file_scheme(src), strip_file_scheme(dst), ec);
  return !ec;
}

int64_t FileMgr::count(const std::string& path) const { return (int64_t)list_info(path).size(); }

FileMgr& default_file_mgr() {
  static FileMgr m;
  return m;
}

}  // namespace pbx
