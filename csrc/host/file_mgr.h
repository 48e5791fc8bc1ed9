// File-system client for pass data and model files.
//
// Contract reproduced (not code): boxps::PaddleFileMgr behind BoxFileMgr
// (box_wrapper.h:1016-1041, box_wrapper.cc:1326-1397) and the dataset's file
// sources fs_open_read / hdfs_open_read with converter pipes and gzip
// (fw/io/fs.h:31-97, fw/io/shell.h:60-73).  The reference links a proprietary
// AFS client; this one serves local paths with POSIX calls and remote
// (hdfs:// / afs://) paths through the cluster's `hadoop fs` command line, the
// way Paddle's own hdfs_* functions do:
//
//   <hadoop_bin> fs -D fs.default.name=<fs_name> -D hadoop.job.ugi=<fs_ugi> -<verb> ...
//
// The pass loader threads (slot_dataset.cc) open every file through
// open_read(), so a filelist may mix local and remote, plain and .gz files.
#pragma once
#include <cstdint>
#include <cstdio>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

namespace pbx {

class FileMgr {
 public:
  // fs_name "" = local only; hadoop_bin defaults to $HADOOP_HOME/bin/hadoop
  // when HADOOP_HOME is set, else "hadoop" on PATH
  bool init(const std::string& fs_name, const std::string& fs_ugi, const std::string& conf_path,
            const std::string& hadoop_bin = "");
  void destroy();

  static bool is_remote(const std::string& path);
  // "hadoop fs -D ... " prefix for remote paths ("" before init)
  std::string remote_prefix() const;

  // stream opened for reading: a FILE* (local, uncompressed, no converter) or
  // a pipe through `cat|zcat|hadoop fs -cat` and the converter command
  FILE* open_read(const std::string& path, const std::string& pipe_command, bool* is_pipe) const;
  FILE* open_write(const std::string& path, bool* is_pipe) const;
  static void close(FILE* f, bool is_pipe);

  std::vector<std::string> list_dir(const std::string& path) const;
  std::vector<std::pair<std::string, int64_t>> list_info(const std::string& path) const;
  bool makedir(const std::string& path) const;
  bool exists(const std::string& path) const;
  bool download(const std::string& remote, const std::string& local) const;
  bool upload(const std::string& local, const std::string& remote) const;
  bool remove(const std::string& path) const;
  int64_t file_size(const std::string& path) const;  // -1 when missing
  // per entry of a directory (or the file itself): (path, bytes incl. subtree)
  std::vector<std::pair<std::string, int64_t>> dus(const std::string& path) const;
  bool truncate(const std::string& path, int64_t len) const;
  bool touch(const std::string& path) const;
  bool rename(const std::string& src, const std::string& dst) const;
  int64_t count(const std::string& path) const;

  // last shell command (debugging / tests)
  std::string last_command() const;

 private:
  int run(const std::string& cmd, std::string* out) const;
  std::string fs_name_, fs_ugi_, conf_path_, hadoop_bin_ = "hadoop";
  bool inited_ = false;
  mutable std::mutex mu_;
  mutable std::string last_cmd_;
};

// process-wide client used by the pass loaders (BoxFileMgr.init configures it)
FileMgr& default_file_mgr();

}  // namespace pbx
