/*
 * device_hip.cpp — the Cycles-side plugin a maintainer adds to
 * intern/cycles/device/ so Blender's unchanged host drives the MI355X path
 * tracer.  It is a ccl::Device (device/device.h:288-500) whose every method
 * forwards to the C ABI of include/hipcycles.h; nothing here computes.
 *
 * Registration (INTEGRATION.md lists the exact edits):
 *   device/device_intern.h   declare device_hipcy_init/create/info
 *   device/device.cpp:385    case DEVICE_HIPCY: device = device_hipcy_create(info, stats, profiler, background);
 *   device/device.cpp:500    append device_hipcy_info(...) in available_devices
 *   device/device.h:43-60    DEVICE_HIPCY in DeviceType / DEVICE_MASK_HIPCY
 *
 * Semantics mirror CUDADevice (device/cuda/device_cuda_impl.cpp):
 *   MEM_GLOBAL arrays are bound by name (global_alloc, :1088-1096);
 *   RENDER tasks loop acquire_tile -> path trace -> update_progress ->
 *   release_tile on one worker thread per device (thread_run, :2342-2391),
 *   the tiles streamed into one running device pass (hipcy_render_feed);
 *   the first error is sticky and reported through error_message().
 *
 * Built and linked with the reference host's own device layer by
 * tools/plugin_harness.sh and driven through DeviceTask RENDER, one or two
 * devices on one tile queue (tests/test_plugin_harness.py); compile-checked
 * against the reference headers by tests/test_integration.py.
 */
#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <deque>
#include <vector>
#include "device/device.h"
#include "device/device_intern.h"

#include "render/buffers.h"

#include "util/util_logging.h"
#include "util/util_string.h"
#include "util/util_task.h"
#include "util/util_thread.h"

#include "hipcycles.h"

CCL_NAMESPACE_BEGIN

/* DEVICE_HIPCY: the DeviceType entry INTEGRATION.md adds after DEVICE_OPTIX
 * (device/device.h:42-50).  Spelled by value so the plugin also builds against
 * an unedited device.h (the harness); never DEVICE_CUDA, whose type checks
 * (device_multi.cpp:112-113, device.cpp:688) would treat this device as CUDA. */
static const DeviceType kDeviceTypeHIPCY = (DeviceType)(DEVICE_OPTIX + 1);

class HIPCyclesDevice : public Device {
 public:
  HIPCyclesDevice(DeviceInfo &info, Stats &stats, Profiler &profiler, bool background)
      : Device(info, stats, profiler, background), dev_(hipcy_create(info.num))
  {
    live_devices_++;
    if (dev_ == nullptr) {
      set_error(string_printf("HIP device %d: %s", info.num, hipcy_global_error()));
    }
    if (const char *env = getenv("CYCLES_HIPCY_STREAM_HOLD")) {
      hold_ = strtoull(env, nullptr, 10);
    }
  }

  ~HIPCyclesDevice() noexcept(false)
  {
    task_pool_.cancel();
    hipcy_destroy(dev_);
    live_devices_--;
  }

  /* device.h:353 — the host keeps building Cycles' BVH2; the device widens it */
  BVHLayoutMask get_bvh_layout_mask() const override
  {
    return BVH_LAYOUT_BVH2;
  }

  /* device.h:366 — KernelData ("__data"), scene.cpp:307 / light.cpp:66 */
  void const_copy_to(const char *name, void *host, size_t size) override
  {
    check(hipcy_const_copy_to(dev_, name, host, size));
  }

  /* device.h:375 — features the kernels do not implement are refused here, and
   * once more against the uploaded KernelData and SVM programs before the first
   * render (hair curves, subsurface scattering, volumes and the shader
   * ray-tracing nodes are implemented; hipcy_load_kernels checks their
   * variants: curve shapes, BSSRDF falloffs, branched path tracing with
   * volumes / BSSRDFs / shadow catchers).  use_shader_raytrace is what
   * ShaderManager::get_requested_features sets for any Ambient Occlusion or
   * Bevel node (render/shader.cpp:724-725): those nodes run on the device. */
  bool load_kernels(const DeviceRequestedFeatures &f) override
  {
    if (f.use_object_motion || f.use_camera_motion || f.use_baking || f.use_patch_evaluation || f.use_denoising) {
      set_error("HIP device: requested features are not implemented (" + f.get_build_options() + ")");
      return false;
    }
    return true;
  }

  /* device.h:484-488 */
  void mem_alloc(device_memory &mem) override
  {
    if (mem.type == MEM_PIXELS) {
      set_error(string_printf("HIP device: memory kind of %s is not supported", mem.name));
      return;
    }
    if (mem.type == MEM_TEXTURE) {
      /* CUDADevice::mem_alloc asserts here too: textures are created by
       * mem_copy_to -> tex_alloc */
      set_error(string_printf("HIP device: mem_alloc of texture %s (use mem_copy_to)", mem.name));
      return;
    }
    uint64_t ptr = 0;
    const size_t bytes = mem.memory_size();
    if (check(hipcy_mem_alloc(dev_, bytes, &ptr))) {
      mem.device_pointer = (device_ptr)ptr;
      mem.device_size = bytes;
      stats.mem_alloc(bytes);
    }
  }

  /* device_cuda_impl.cpp:1105-1304 tex_alloc: the device copies the texels and
   * keeps TextureInfo[slot] in its own __texture_info table */
  void tex_alloc(device_texture &mem)
  {
    /* 3D textures (data_depth > 1: volume grids, Point Density voxels) keep
     * their TextureInfo 3D transform (util_texture.h:93-107) */
    const float *tfm3d = mem.info.use_transform_3d ? (const float *)&mem.info.transform_3d : nullptr;
    if (check(hipcy_tex_alloc_3d(dev_, (int)mem.slot, (int)mem.info.data_type, (int)mem.info.interpolation,
                                 (int)mem.info.extension, (int)mem.data_width,
                                 (int)std::max<size_t>(mem.data_height, 1), (int)std::max<size_t>(mem.data_depth, 1),
                                 tfm3d, mem.host_pointer, mem.memory_size()))) {
      mem.device_pointer = (device_ptr)(mem.slot + 1); /* a token: the device owns the texels */
      mem.device_size = mem.memory_size();
      stats.mem_alloc(mem.device_size);
    }
  }

  void tex_free(device_texture &mem)
  {
    if (mem.device_pointer) {
      hipcy_tex_free(dev_, (int)mem.slot);
      stats.mem_free(mem.device_size);
      mem.device_pointer = 0;
      mem.device_size = 0;
    }
  }

  void mem_copy_to(device_memory &mem) override
  {
    if (mem.type == MEM_TEXTURE) {
      tex_free((device_texture &)mem);
      tex_alloc((device_texture &)mem);
      return;
    }
    if (!mem.device_pointer) {
      mem_alloc(mem);
    }
    if (!mem.device_pointer) {
      return;
    }
    if (mem.host_pointer && mem.memory_size()) {
      check(hipcy_mem_copy_to(dev_, (uint64_t)mem.device_pointer, mem.host_pointer, mem.memory_size()));
    }
    if (mem.type == MEM_GLOBAL) {
      /* CUDADevice::global_alloc: bind the array to its kernel_textures.h name */
      check(hipcy_bind_global(dev_, mem.name, (uint64_t)mem.device_pointer, mem.memory_size()));
    }
  }

  void mem_copy_from(device_memory &mem, int y, int w, int h, int elem) override
  {
    const size_t offset = (size_t)elem * y * w;
    const size_t size = (size_t)elem * w * h;
    if (mem.host_pointer && mem.device_pointer) {
      check(hipcy_mem_copy_from(dev_, (char *)mem.host_pointer + offset, (uint64_t)mem.device_pointer + offset,
                                size));
    }
  }

  void mem_zero(device_memory &mem) override
  {
    if (!mem.device_pointer) {
      mem_alloc(mem);
    }
    if (mem.host_pointer) {
      memset(mem.host_pointer, 0, mem.memory_size());
    }
    if (mem.device_pointer) {
      check(hipcy_mem_zero(dev_, (uint64_t)mem.device_pointer, mem.memory_size()));
    }
  }

  void mem_free(device_memory &mem) override
  {
    if (mem.type == MEM_TEXTURE) {
      tex_free((device_texture &)mem);
      return;
    }
    if (mem.device_pointer) {
      if (mem.type == MEM_GLOBAL) {
        hipcy_bind_global(dev_, mem.name, 0, 0);
      }
      check(hipcy_mem_free(dev_, (uint64_t)mem.device_pointer));
      stats.mem_free(mem.device_size);
      mem.device_pointer = 0;
      mem.device_size = 0;
    }
  }

  /* device.h:403-405 — one worker thread per device, like CUDADevice::task_add */
  void task_add(DeviceTask &task) override
  {
    if (task.type == DeviceTask::FILM_CONVERT) {
      /* on the calling thread, like CUDADevice::task_add (device_cuda_impl.cpp:2427-2430)
       * -> film_convert (:1954-2017) */
      check(hipcy_film_convert(dev_, (uint64_t)task.buffer, (uint64_t)task.rgba_byte, (uint64_t)task.rgba_half,
                               1.0f / (task.sample + 1), task.x, task.y, task.w, task.h, task.offset,
                               task.stride));
      return;
    }
    if (task.type == DeviceTask::SHADER) {
      /* LightManager background map (light.cpp:38-85) and MeshManager::displace
       * (mesh_displace.cpp, SHADER_EVAL_DISPLACE) -> CUDADevice::shader
       * (device_cuda_impl.cpp:2019-2093) */
      task_pool_.push([=] {
        /* per sample, 64K-pixel chunks with a cancel check between them and
         * progress after each sample, as CUDADevice::shader does; neither
         * evaluation depends on the sample index (kernel_bake.h:446-510) */
        DeviceTask task_copy = task;
        const int chunk = 0x10000;
        const int end = task.shader_x + task.shader_w;
        for (int sample = 0; sample < task.num_samples; sample++) {
          for (int x = task.shader_x; x < end; x += chunk) {
            if (task_copy.get_cancel()) {
              return;
            }
            check(hipcy_shader_eval(dev_, (int)task.shader_eval_type, (uint64_t)task.shader_input,
                                    (uint64_t)task.shader_output, x, std::min(chunk, end - x), task.offset, 1));
          }
          task_copy.update_progress(NULL);
        }
      });
      return;
    }
    if (task.type != DeviceTask::RENDER) {
      set_error("HIP device: only RENDER, SHADER and FILM_CONVERT tasks are implemented");
      return;
    }
    task_pool_.push([=] {
      DeviceTask task_copy = task;
      render(task_copy);
    });
  }

  void task_wait() override
  {
    task_pool_.wait();
  }

  void task_cancel() override
  {
    task_pool_.cancel();
  }

 private:
  hipcy_device *dev_;
  DedicatedTaskPool task_pool_; /* one worker thread, as CUDADevice (device_cuda.h:45) */
  /* pixel-samples a RENDER task may hold; CYCLES_HIPCY_STREAM_HOLD overrides
   * the choice of stream_hold() */
  uint64_t hold_ = 0;
  /* HIPCyclesDevice instances alive in this process: the sub-devices of one
   * MultiDevice (device_multi.cpp:47-105 creates them all before any task) */
  static std::atomic<int> live_devices_;

  /* How much of the session's tile queue one RENDER task may hold, in
   * pixel-samples (0: the device default, its whole slot pool in flight plus as
   * much in reserve).  The only device of the session takes the default, so a
   * frame renders in as few wavefront iterations as a whole-frame pass.
   * Devices sharing one TileManager queue (MultiDevice, device_multi.cpp:689-737)
   * hold a fair part of the frame: the first tile's RenderBuffers tell the frame
   * (BufferParams full_width x full_height at the tile's resolution divider,
   * times the tile's sample count; buffers.h:38-50), and each of the
   * live_devices_ devices holds CYCLES_HIPCY_HOLD_SHARE (default 1/2) of its
   * 1/N of it: half the frame is dealt out by the first fills, the other half
   * goes to whichever device runs low first, so devices that start late or
   * draw expensive tiles still finish together.  Without RenderBuffers on the
   * tile the hold is 2^25 pixel-samples (64 tiles of 64x64 at 128 spp). */
  uint64_t stream_hold(const RenderTile *first) const
  {
    if (hold_) {
      return hold_;
    }
    const int live = live_devices_.load();
    if (live <= 1) {
      return 0;
    }
    if (first == nullptr || first->buffers == nullptr) {
      return (uint64_t)1 << 25;
    }
    const BufferParams &p = first->buffers->params;
    const uint64_t res = (uint64_t)std::max(first->resolution, 1);
    const uint64_t frame = (uint64_t)std::max(p.full_width, p.width) * (uint64_t)std::max(p.full_height, p.height) /
                           (res * res) * (uint64_t)std::max(first->num_samples, 1);
    double share = 0.5;
    if (const char *env = getenv("CYCLES_HIPCY_HOLD_SHARE")) {
      share = std::min(std::max(atof(env), 0.05), 1.0);
    }
    const uint64_t tile = (uint64_t)first->w * first->h * (uint64_t)std::max(first->num_samples, 1);
    return std::max<uint64_t>((uint64_t)(share * (double)frame / live), tile);
  }

  bool check(int rc)
  {
    if (rc != 0 && dev_ != nullptr) {
      set_error(string_printf("HIP device: %s", hipcy_error(dev_)));
    }
    return rc == 0;
  }

  /* CUDADevice::thread_run RENDER branch (device_cuda_impl.cpp:2346-2386):
   * acquire_tile -> render -> update_progress -> release_tile, with the tiles
   * streamed into one running device pass (hipcy_render_feed).  The device
   * asks for a tile only when its unclaimed work runs low and never holds more
   * than `hold` pixel-samples, so devices sharing the session's TileManager
   * queue (MultiDevice::task_add, device_multi.cpp:689-737, one cloned task per
   * device) each take tiles as fast as they finish them; every tile is
   * released as soon as all of its samples are in its buffer. */
  struct Feed {
    HIPCyclesDevice *self;
    DeviceTask *task;
    std::deque<RenderTile> tiles; /* acquired, indexed by the feed tag */
    bool have_first = false;      /* the tile render() acquired to size the hold */
    RenderTile first;
  };

  /* the next PATH_TRACE tile of the queue (others are released unrendered) */
  static bool next_tile(Feed *f, RenderTile &tile)
  {
    if (f->have_first) {
      f->have_first = false;
      tile = f->first;
      return true;
    }
    DeviceTask &task = *f->task;
    while (task.acquire_tile(f->self, tile, task.tile_types)) {
      if (tile.task == RenderTile::PATH_TRACE) {
        return true;
      }
      task.release_tile(tile);
    }
    return false;
  }

  static int feed_acquire(void *user, hipcy_work_tile *wt, uint64_t *tag)
  {
    Feed *f = (Feed *)user;
    RenderTile tile;
    if (!next_tile(f, tile)) {
      return 0;
    }
    wt->x = tile.x;
    wt->y = tile.y;
    wt->w = tile.w;
    wt->h = tile.h;
    wt->start_sample = tile.start_sample;
    wt->num_samples = tile.num_samples;
    wt->offset = tile.offset;
    wt->stride = tile.stride;
    wt->buffer = (uint64_t)tile.buffer;
    *tag = f->tiles.size();
    f->tiles.push_back(tile);
    return 1;
  }

  /* every acquired tile comes back here once: finished, or (after a device
   * error, hipcy_error non-empty) unfinished, released without progress as
   * CUDADevice::thread_run still releases a tile whose render failed */
  static void feed_release(void *user, const hipcy_work_tile *, uint64_t tag)
  {
    Feed *f = (Feed *)user;
    RenderTile &t = f->tiles[tag];
    if (hipcy_error(f->self->dev_)[0] == '\0') {
      t.sample = t.start_sample + t.num_samples;
      f->task->update_progress(&t, t.w * t.h * t.num_samples);
    }
    f->task->release_tile(t);
  }

  static int feed_cancelled(void *user)
  {
    Feed *f = (Feed *)user;
    return f->task->get_cancel() && !f->task->need_finish_queue;
  }

  void render(DeviceTask &task)
  {
    if (!check(hipcy_load_kernels(dev_))) {
      return;
    }
    Feed f;
    f.self = this;
    f.task = &task;
    /* the first tile sizes the hold; it is the first one the feed renders */
    f.have_first = next_tile(&f, f.first);
    if (!f.have_first) {
      return;
    }
    f.have_first = true;
    hipcy_tile_feed feed;
    feed.user = &f;
    feed.acquire = feed_acquire;
    feed.release = feed_release;
    feed.cancelled = feed_cancelled;
    feed.hold = stream_hold(&f.first);
    check(hipcy_render_feed(dev_, &feed));
    if (f.have_first) {
      /* the feed failed before it took the first tile: hand it back unrendered */
      f.have_first = false;
      task.release_tile(f.first);
    }
  }
};

std::atomic<int> HIPCyclesDevice::live_devices_{0};

bool device_hipcy_init()
{
  int n = 0;
  return hipcy_device_count(&n) == 0 && n > 0;
}

Device *device_hipcy_create(DeviceInfo &info, Stats &stats, Profiler &profiler, bool background)
{
  return new HIPCyclesDevice(info, stats, profiler, background);
}

void device_hipcy_info(vector<DeviceInfo> &devices)
{
  int n = 0;
  hipcy_device_count(&n);
  for (int i = 0; i < n; i++) {
    char name[256];
    uint64_t mem = 0;
    if (hipcy_device_info(i, name, sizeof(name), &mem) != 0) {
      continue;
    }
    DeviceInfo info;
    info.type = kDeviceTypeHIPCY;
    info.description = string(name);
    info.num = i;
    info.id = string_printf("HIPCY_%d", i);
    info.has_half_images = false;
    info.has_volume_decoupled = false;
    info.has_osl = false;
    info.has_profiling = false;
    info.denoisers = DENOISER_NONE;
    devices.push_back(info);
  }
}

CCL_NAMESPACE_END
