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
 * usage: plugin_harness <scene dir> <width> <height> <samples> <tile size> <pass stride> <out.bin>
 * The scene dir holds kernel_data.bin, manifest.txt ("name bytes" lines) and
 * one <name>.bin per array (written by tests/test_plugin_harness.py).
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

int main(int argc, char **argv)
{
  if (argc != 8) {
    fprintf(stderr, "usage: %s dir width height samples tile pass_stride out.bin\n", argv[0]);
    return 2;
  }
  const std::string dir = argv[1];
  const int W = atoi(argv[2]), H = atoi(argv[3]), S = atoi(argv[4]), T = atoi(argv[5]), stride = atoi(argv[6]);

  if (!device_hipcy_init()) {
    fprintf(stderr, "no HIP device\n");
    return 3;
  }
  vector<DeviceInfo> infos;
  device_hipcy_info(infos);
  Stats stats;
  Profiler profiler;
  Device *dev = device_hipcy_create(infos[0], stats, profiler, true);
  if (dev->have_error()) {
    fprintf(stderr, "create: %s\n", dev->error_message().c_str());
    return 4;
  }
  printf("device: %s (%s)\n", infos[0].description.c_str(), infos[0].id.c_str());
  DeviceRequestedFeatures features;
  if (!dev->load_kernels(features)) {
    fprintf(stderr, "load_kernels: %s\n", dev->error_message().c_str());
    return 4;
  }

  /* scene arrays, bound by name (MEM_GLOBAL) */
  std::vector<device_vector<uchar> *> arrays;
  std::vector<std::string> names;
  {
    std::ifstream man(dir + "/manifest.txt");
    std::string name;
    size_t bytes;
    while (man >> name >> bytes) {
      names.push_back(name);
    }
  }
  {
    std::ifstream man(dir + "/manifest.txt");
    std::string name;
    size_t bytes;
    size_t i = 0;
    while (man >> name >> bytes) {
      auto *v = new device_vector<uchar>(dev, names[i++].c_str(), MEM_GLOBAL);
      uchar *p = v->alloc(bytes);
      if (!read_file(dir + "/" + name + ".bin", p, bytes)) {
        fprintf(stderr, "short read: %s\n", name.c_str());
        return 5;
      }
      v->copy_to_device();
      arrays.push_back(v);
    }
  }
  std::vector<char> kd(1 << 16);
  std::ifstream kf(dir + "/kernel_data.bin", std::ios::binary);
  kf.read(kd.data(), (std::streamsize)kd.size());
  dev->const_copy_to("__data", kd.data(), (size_t)kf.gcount());

  device_vector<float> buffer(dev, "render_buffer", MEM_READ_WRITE);
  buffer.alloc((size_t)W * H * stride);
  buffer.zero_to_device();

  /* the TileManager's role: tiles in row order, each rendered with all samples */
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
      t.buffer = buffer.device_pointer;
      tiles.push_back(t);
    }
  }
  std::mutex mtx;
  size_t next = 0, released = 0;
  long progress = 0;
  DeviceTask task(DeviceTask::RENDER);
  task.acquire_tile = [&](Device *, RenderTile &tile, uint tile_types) {
    std::lock_guard<std::mutex> lock(mtx);
    if (next >= tiles.size() || !(tile_types & RenderTile::PATH_TRACE)) {
      return false;
    }
    tile = tiles[next++];
    return true;
  };
  task.release_tile = [&](RenderTile &tile) {
    std::lock_guard<std::mutex> lock(mtx);
    if (tile.sample != tile.start_sample + tile.num_samples) {
      fprintf(stderr, "tile %d released at sample %d\n", tile.tile_index, tile.sample);
    }
    released++;
  };
  task.update_progress_sample = [&](long pixel_samples, int) { progress += pixel_samples; };
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
  task.buffer = buffer.device_pointer;
  task.pass_stride = stride;

  dev->task_add(task);
  dev->task_wait();
  if (dev->have_error()) {
    fprintf(stderr, "render: %s\n", dev->error_message().c_str());
    return 6;
  }
  buffer.copy_from_device(0, W * stride, H);
  printf("tiles %zu released %zu progress %ld pixel-samples\n", tiles.size(), released, progress);
  if (released != tiles.size() || progress != (long)W * H * S) {
    fprintf(stderr, "tile bookkeeping mismatch\n");
    return 7;
  }
  FILE *out = fopen(argv[7], "wb");
  fwrite(buffer.data(), sizeof(float), (size_t)W * H * stride, out);
  fclose(out);

  for (auto *v : arrays) {
    v->free();
    delete v;
  }
  buffer.free();
  delete dev;
  return 0;
}
