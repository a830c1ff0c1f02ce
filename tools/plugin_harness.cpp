/*
 * plugin_harness.cpp — drives integration/device_hip.cpp (the ccl::Device
 * plugin) through the reference host's own device-layer classes, linked from
 * the reference sources (tools/plugin_harness.sh builds it): ccl::Device
 * (device/device.cpp), device_memory / device_vector (device_memory.cpp),
 * DeviceTask (device_task.cpp), RenderTile (render/buffers.cpp) and the util
 * task pool / threads.  Test infrastructure: it is never part of the product.
 *
 * What it does is what render/session.cpp does with a GPU device for one
 * frame (Session::run_gpu -> DeviceTask RENDER, session.cpp:381-533):
 *   device_hipcy_info / device_hipcy_create      (device.cpp:367-418 path)
 *   MEM_GLOBAL device_vector uploads by name     (scene.cpp device_update)
 *   const_copy_to("__data", KernelData)
 *   a MEM_READ_WRITE render buffer, zeroed
 *   DeviceTask RENDER whose acquire_tile hands out tile_size tiles (the
 *   TileManager's role) until the frame is done; release_tile counts them
 *   task_add / task_wait, then mem_copy_from of the buffer
 *
 * usage: plugin_harness <scene dir> <width> <height> <samples> <tile size> <pass stride> <out.bin> [devices]
 * The scene dir holds kernel_data.bin, manifest.txt ("name bytes" lines) and
 * one <name>.bin per array (written by tests/test_plugin_harness.py).
 *
 * With devices > 1 it does what MultiDevice does (device_multi.cpp:689-737):
 * one HIPCyclesDevice per sub-device, each with its own scene upload and
 * render buffer, each given a clone of the RENDER task (DeviceTask::split of a
 * RENDER task copies it), all acquiring from the one shared tile queue; a tile
 * is rendered into the buffer of the device that acquired it, and the frame
 * is assembled from the tiles each device released.  Prints the tiles each
 * device rendered.  The sub-devices share GPU 0 here (one-GPU test box).
 */
#include <cstdio>
#include <cstring>
#include <fstream>
#include <mutex>
#include <string>
#include <vector>

#include "device/device.h"
#include "device/device_memory.h"
#include "device/device_task.h"
#include "render/buffers.h"
#include "util/util_profiling.h"
#include "util/util_stats.h"
#include "util/util_time.h"

CCL_NAMESPACE_BEGIN
bool device_hipcy_init();
Device *device_hipcy_create(DeviceInfo &info, Stats &stats, Profiler &profiler, bool background);
void device_hipcy_info(vector<DeviceInfo> &devices);
CCL_NAMESPACE_END

using namespace ccl;

static bool read_file(const std::string &path, void *dst, size_t bytes)
{
  std::ifstream f(path, std::ios::binary);
  f.read((char *)dst, (std::streamsize)bytes);
  return (size_t)f.gcount() == bytes;
}

struct SubDevice {
  Device *dev = nullptr;
  std::vector<device_vector<uchar> *> arrays;
  device_vector<float> *buffer = nullptr;
  std::vector<int> tiles; /* indices of the tiles it acquired */
  int held = 0;           /* acquired and not yet released */
  int max_held = 0;
};

static int upload_scene(SubDevice &sd, const std::string &dir, int W, int H, int stride)
{
  std::vector<std::string> names;
  std::vector<size_t> sizes;
  {
    std::ifstream man(dir + "/manifest.txt");
    std::string name;
    size_t bytes;
    while (man >> name >> bytes) {
      names.push_back(name);
      sizes.push_back(bytes);
    }
  }
  for (size_t i = 0; i < names.size(); i++) {
    auto *v = new device_vector<uchar>(sd.dev, names[i].c_str(), MEM_GLOBAL);
    uchar *p = v->alloc(sizes[i]);
    if (!read_file(dir + "/" + names[i] + ".bin", p, sizes[i])) {
      fprintf(stderr, "short read: %s\n", names[i].c_str());
      return 5;
    }
    v->copy_to_device();
    sd.arrays.push_back(v);
  }
  std::vector<char> kd(1 << 16);
  std::ifstream kf(dir + "/kernel_data.bin", std::ios::binary);
  kf.read(kd.data(), (std::streamsize)kd.size());
  sd.dev->const_copy_to("__data", kd.data(), (size_t)kf.gcount());
  sd.buffer = new device_vector<float>(sd.dev, "render_buffer", MEM_READ_WRITE);
  sd.buffer->alloc((size_t)W * H * stride);
  sd.buffer->zero_to_device();
  return 0;
}

int main(int argc, char **argv)
{
  if (argc != 8 && argc != 9) {
    fprintf(stderr, "usage: %s dir width height samples tile pass_stride out.bin [devices]\n", argv[0]);
    return 2;
  }
  const std::string dir = argv[1];
  const int W = atoi(argv[2]), H = atoi(argv[3]), S = atoi(argv[4]), T = atoi(argv[5]), stride = atoi(argv[6]);
  const int ndev = argc == 9 ? atoi(argv[8]) : 1;

  if (!device_hipcy_init()) {
    fprintf(stderr, "no HIP device\n");
    return 3;
  }
  vector<DeviceInfo> infos;
  device_hipcy_info(infos);
  Stats stats;
  Profiler profiler;
  std::vector<SubDevice> subs(ndev);
  for (int d = 0; d < ndev; d++) {
    subs[d].dev = device_hipcy_create(infos[0], stats, profiler, true);
    if (subs[d].dev->have_error()) {
      fprintf(stderr, "create: %s\n", subs[d].dev->error_message().c_str());
      return 4;
    }
    DeviceRequestedFeatures features;
    if (!subs[d].dev->load_kernels(features)) {
      fprintf(stderr, "load_kernels: %s\n", subs[d].dev->error_message().c_str());
      return 4;
    }
    const int rc = upload_scene(subs[d], dir, W, H, stride);
    if (rc) {
      return rc;
    }
  }
  printf("device: %s (%s) x %d\n", infos[0].description.c_str(), infos[0].id.c_str(), ndev);

  /* the TileManager's role: tiles in row order, each rendered with all
   * samples, handed out from one queue to whichever device asks */
  std::vector<RenderTile> tiles;
  for (int y = 0; y < H; y += T) {
    for (int x = 0; x < W; x += T) {
      RenderTile t;
      t.task = RenderTile::PATH_TRACE;
      t.x = x;
      t.y = y;
      t.w = std::min(T, W - x);
      t.h = std::min(T, H - y);
      t.start_sample = 0;
      t.num_samples = S;
      t.sample = 0;
      t.resolution = 1;
      t.offset = 0;
      t.stride = W;
      t.tile_index = (int)tiles.size();
      tiles.push_back(t);
    }
  }
  std::mutex mtx;
  size_t next = 0, released = 0;
  long progress = 0;
  std::vector<int> done(tiles.size(), 0);
  std::vector<double> t_last(ndev, 0.0);
  const double t_start = time_dt();
  DeviceTask task(DeviceTask::RENDER);
  task.acquire_tile = [&](Device *dev, RenderTile &tile, uint tile_types) {
    std::lock_guard<std::mutex> lock(mtx);
    if (next >= tiles.size() || !(tile_types & RenderTile::PATH_TRACE)) {
      return false;
    }
    for (SubDevice &sd : subs) {
      if (sd.dev == dev) {
        tile = tiles[next];
        tile.buffer = sd.buffer->device_pointer;
        sd.tiles.push_back((int)next);
        next++;
        sd.max_held = std::max(sd.max_held, ++sd.held);
        return true;
      }
    }
    return false;
  };
  task.release_tile = [&](RenderTile &tile) {
    std::lock_guard<std::mutex> lock(mtx);
    if (tile.sample != tile.start_sample + tile.num_samples) {
      fprintf(stderr, "tile %d released at sample %d\n", tile.tile_index, tile.sample);
    }
    done[tile.tile_index]++;
    released++;
    for (size_t d = 0; d < subs.size(); d++) {
      if (tile.buffer == subs[d].buffer->device_pointer) {
        t_last[d] = time_dt() - t_start;
        subs[d].held--;
      }
    }
  };
  task.update_progress_sample = [&](long pixel_samples, int) {
    std::lock_guard<std::mutex> lock(mtx);
    progress += pixel_samples;
  };
  task.update_tile_sample = [&](RenderTile &) {};
  task.get_cancel = [] { return false; };
  task.tile_types = RenderTile::PATH_TRACE;
  task.need_finish_queue = false;
  task.num_samples = S;
  task.sample = 0;
  task.x = 0;
  task.y = 0;
  task.w = W;
  task.h = H;
  task.offset = 0;
  task.stride = W;
  task.pass_stride = stride;

  /* MultiDevice::task_add: a clone of the task per sub-device, then task_wait */
  for (SubDevice &sd : subs) {
    DeviceTask subtask = task;
    subtask.buffer = sd.buffer->device_pointer;
    sd.dev->task_add(subtask);
  }
  for (SubDevice &sd : subs) {
    sd.dev->task_wait();
    if (sd.dev->have_error()) {
      fprintf(stderr, "render: %s\n", sd.dev->error_message().c_str());
      return 6;
    }
  }
  std::vector<float> film((size_t)W * H * stride, 0.0f);
  for (int d = 0; d < ndev; d++) {
    SubDevice &sd = subs[d];
    sd.buffer->copy_from_device(0, W * stride, H);
    for (int k : sd.tiles) {
      const RenderTile &t = tiles[k];
      for (int y = t.y; y < t.y + t.h; y++) {
        memcpy(&film[((size_t)y * W + t.x) * stride], &sd.buffer->data()[((size_t)y * W + t.x) * stride],
               sizeof(float) * t.w * stride);
      }
    }
    printf("device %d tiles %zu max held %d last release %.3f s\n", d, sd.tiles.size(), sd.max_held, t_last[d]);
  }
  bool once = true;
  for (int c : done) {
    once &= c == 1;
  }
  printf("tiles %zu released %zu progress %ld pixel-samples\n", tiles.size(), released, progress);
  if (released != tiles.size() || !once || progress != (long)W * H * S) {
    fprintf(stderr, "tile bookkeeping mismatch\n");
    return 7;
  }
  FILE *out = fopen(argv[7], "wb");
  fwrite(film.data(), sizeof(float), film.size(), out);
  fclose(out);

  for (SubDevice &sd : subs) {
    for (auto *v : sd.arrays) {
      v->free();
      delete v;
    }
    sd.buffer->free();
    delete sd.buffer;
    delete sd.dev;
  }
  return 0;
}
