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
 *   load_kernels(DeviceRequestedFeatures)        (session.cpp load_kernels; features.txt
 *                                                 sets use_shader_raytrace as shader.cpp:724-725
 *                                                 does for AO / Bevel nodes)
 *   MEM_GLOBAL device_vector uploads by name     (scene.cpp device_update)
 *   MEM_TEXTURE device_texture uploads           (image.cpp device_load_image: textures.txt)
 *   const_copy_to("__data", KernelData)
 *   the background importance map: a DeviceTask SHADER with
 *   SHADER_EVAL_BACKGROUND over the map (light.cpp:38-85 shade_background_pixels,
 *   split in 128x128-element tasks), its CDFs built on the host
 *   (libhipcycles_host.so, light.cpp:530-716) and re-uploaded (background.txt)
 *   a MEM_READ_WRITE render buffer, zeroed
 *   DeviceTask RENDER whose acquire_tile hands out tile_size tiles (the
 *   TileManager's role) until the frame is done; release_tile counts them
 *   task_add / task_wait, then mem_copy_from of the buffer
 *
 * usage: plugin_harness <scene dir> <width> <height> <samples> <tile size> <pass stride> <out.bin> [devices]
 * The scene dir holds kernel_data.bin, manifest.txt ("name bytes" lines) and
 * one <name>.bin per array (written by tests/test_plugin_harness.py), and
 * optionally textures.txt ("slot data_type interpolation extension width
 * height" lines, texels in tex_<slot>.bin), background.txt ("res_x res_y")
 * and features.txt ("name 0|1" lines of DeviceRequestedFeatures).
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
#include "util/util_math.h"
#include "util/util_profiling.h"
#include "util/util_stats.h"
#include "util/util_time.h"

CCL_NAMESPACE_BEGIN
bool device_hipcy_init();
Device *device_hipcy_create(DeviceInfo &info, Stats &stats, Profiler &profiler, bool background);
void device_hipcy_info(vector<DeviceInfo> &devices);
CCL_NAMESPACE_END

/* the repository's host restatement of the background CDFs (render/light.cpp
 * background_cdf), csrc/host/light_background.cpp in libhipcycles_host.so */
extern "C" void hcb_background_cdf(const float *pixels, int res_x, int res_y, float *marg_cdf, float *cond_cdf);

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
  std::vector<device_texture *> textures;
  device_vector<float> *buffer = nullptr;
  std::vector<int> tiles; /* indices of the tiles it acquired */
  int held = 0;           /* acquired and not yet released */
  int max_held = 0;
};

static device_vector<uchar> *find_array(SubDevice &sd, const char *name)
{
  for (auto *v : sd.arrays) {
    if (strcmp(v->name, name) == 0) {
      return v;
    }
  }
  auto *v = new device_vector<uchar>(sd.dev, name, MEM_GLOBAL);
  sd.arrays.push_back(v);
  return v;
}

/* shade_background_pixels (light.cpp:38-85): the world shader over the map by
 * DeviceTask SHADER, split in 128x128-element tasks (DeviceTask::split of
 * SHADER tasks), each task_add / task_wait / copy_from_device; then the CDFs on
 * the host and the two CDF arrays re-uploaded by name. */
static int shade_background(SubDevice &sd, int width, int height)
{
  Device *device = sd.dev;
  device_vector<uint4> d_input(device, "background_input", MEM_READ_ONLY);
  device_vector<float4> d_output(device, "background_output", MEM_READ_WRITE);
  uint4 *in = d_input.alloc((size_t)width * height);
  for (int y = 0; y < height; y++) {
    for (int x = 0; x < width; x++) {
      const float u = (x + 0.5f) / width;
      const float v = (y + 0.5f) / height;
      in[x + y * width] = make_uint4(__float_as_uint(u), __float_as_uint(v), 0, 0);
    }
  }
  d_output.alloc((size_t)width * height);
  d_output.zero_to_device();
  d_input.copy_to_device();
  DeviceTask main_task(DeviceTask::SHADER);
  main_task.shader_input = d_input.device_pointer;
  main_task.shader_output = d_output.device_pointer;
  main_task.shader_eval_type = SHADER_EVAL_BACKGROUND;
  main_task.shader_x = 0;
  main_task.shader_w = width * height;
  main_task.num_samples = 1;
  main_task.get_cancel = [] { return false; };
  main_task.update_progress_sample = [](long, int) {};
  list<DeviceTask> split_tasks;
  main_task.split(split_tasks, 1, 128 * 128);
  int n_tasks = 0;
  for (DeviceTask &task : split_tasks) {
    device->task_add(task);
    device->task_wait();
    d_output.copy_from_device(task.shader_x, 1, task.shader_w);
    n_tasks++;
  }
  if (device->have_error()) {
    fprintf(stderr, "background SHADER task: %s\n", device->error_message().c_str());
    return 8;
  }
  d_input.free();
  std::vector<float> pixels((size_t)4 * width * height);
  memcpy(pixels.data(), d_output.data(), pixels.size() * sizeof(float));
  d_output.free();
  std::vector<float> marg((size_t)2 * (height + 1)), cond((size_t)2 * (width + 1) * height);
  hcb_background_cdf(pixels.data(), width, height, marg.data(), cond.data());
  const std::pair<const char *, std::vector<float> *> cdfs[2] = {{"__light_background_marginal_cdf", &marg},
                                                                 {"__light_background_conditional_cdf", &cond}};
  for (const auto &c : cdfs) {
    device_vector<uchar> *v = find_array(sd, c.first);
    uchar *p = v->alloc(c.second->size() * sizeof(float));
    memcpy(p, c.second->data(), c.second->size() * sizeof(float));
    v->copy_to_device();
  }
  printf("background map %dx%d by %d SHADER task(s)\n", width, height, n_tasks);
  return 0;
}

static DeviceRequestedFeatures read_features(const std::string &dir)
{
  DeviceRequestedFeatures f;
  std::ifstream ff(dir + "/features.txt");
  std::string name;
  int on;
  while (ff >> name >> on) {
    if (name == "shader_raytrace") f.use_shader_raytrace = on != 0;
    else if (name == "hair") f.use_hair = on != 0;
    else if (name == "volume") f.use_volume = on != 0;
    else if (name == "subsurface") f.use_subsurface = on != 0;
    else if (name == "transparent") f.use_transparent = on != 0;
    else if (name == "background_light") f.use_background_light = on != 0;
    else fprintf(stderr, "features.txt: unknown feature %s\n", name.c_str());
  }
  return f;
}

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
  {
    /* ImageManager::device_load_image: a device_texture per slot, copy_to_device
     * (-> Device::mem_copy_to -> tex_alloc) */
    std::ifstream tx(dir + "/textures.txt");
    int slot, type, interp, ext;
    size_t w, h;
    while (tx >> slot >> type >> interp >> ext >> w >> h) {
      auto *t = new device_texture(sd.dev, "__tex_image", (uint)slot, (ImageDataType)type, (InterpolationType)interp,
                                   (ExtensionType)ext);
      void *p = t->alloc(w, h);
      if (!read_file(dir + "/tex_" + std::to_string(slot) + ".bin", p, t->memory_size())) {
        fprintf(stderr, "short read: texture %d\n", slot);
        return 5;
      }
      t->copy_to_device();
      sd.textures.push_back(t);
    }
  }
  std::vector<char> kd(1 << 16);
  std::ifstream kf(dir + "/kernel_data.bin", std::ios::binary);
  kf.read(kd.data(), (std::streamsize)kd.size());
  sd.dev->const_copy_to("__data", kd.data(), (size_t)kf.gcount());
  {
    std::ifstream bg(dir + "/background.txt");
    int res_x = 0, res_y = 0;
    if (bg >> res_x >> res_y) {
      /* LightManager::device_update_background (light.cpp:568-716) */
      const int rc = shade_background(sd, res_x, res_y);
      if (rc) {
        return rc;
      }
    }
  }
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
    const DeviceRequestedFeatures features = read_features(dir);
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
  /* Session::acquire_tile hands out tiles with the RenderBuffers whose
   * BufferParams describe the frame (full_width x full_height); the plugin sizes
   * its share of the queue from them */
  RenderBuffers *frame_buffers = new RenderBuffers(subs[0].dev);
  frame_buffers->params.width = frame_buffers->params.full_width = W;
  frame_buffers->params.height = frame_buffers->params.full_height = H;
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
      t.buffers = frame_buffers;
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

  delete frame_buffers;
  for (SubDevice &sd : subs) {
    for (auto *v : sd.arrays) {
      v->free();
      delete v;
    }
    for (auto *t : sd.textures) {
      delete t;
    }
    sd.buffer->free();
    delete sd.buffer;
    delete sd.dev;
  }
  return 0;
}
