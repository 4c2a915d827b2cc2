// Cli.cpp — the `LocoMouse` executable: the same
// command line, files, output and exit codes as the reference's CLI, over the
// host mirror and the MI355X C-ABI.
//
//   LocoMouse <method> config.yml video.avi background.png model.yml calibration.yml L|R output_folder
//
// Reference: main.cpp:38-105 (sequence, messages, exit codes),
// LocoMouse_ParseInputs.cpp:1-99 (arguments, calibration file),
// LocoMouse_class.cpp:12-249 (config.yml), :294-540 (constructor: video,
// background, sizes, flip, output file), :3095-3162 (model file).
#include <algorithm>
#include <chrono>
#include <cmath>
#include <atomic>
#include <cstring>
#include <thread>
#include <cstdlib>
#include <iostream>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "FileStorage.hpp"
#include "LocoMouse.hpp"
#include "Media.hpp"

namespace locomouse {
namespace {

struct ParsedInputs {  // LocoMouse_ParseInputs
  std::string LM_CALL, CONFIG_FILE, VIDEO_FILE, BKG_FILE, MODEL_FILE, CALIBRATION_FILE, FLIP_CHAR, OUTPUT_PATH,
      METHOD, REF_PATH, FILE_STEM;
  std::vector<int32_t> CALIBRATION;
  int calib_rows = 0, calib_cols = 0;
  lm_rect BB_SIDE_VIEW{}, BB_BOTTOM_VIEW{};
};

std::string dir_of(const std::string& p) {  // dirname(3)
  size_t i = p.find_last_of('/');
  if (i == std::string::npos) return ".";
  if (i == 0) return "/";
  return p.substr(0, i);
}

std::string strip_file_name(const std::string& s) {  // ParseInputs.cpp stripFileName
  std::string out;
  size_t i = s.rfind('/');
  if (i != std::string::npos) out = s.substr(i + 1);
  return out.substr(0, out.find_last_of('.'));
}

ParsedInputs parse_inputs(int argc, char** argv) {
  ParsedInputs in;
  in.LM_CALL = argv[0];
  if (argc != 9) {
    std::cout << "Warning: Invalid input list. The input should be: LocoMouse method config.yml video.avi "
                 "background.png model_file.yml calibration_file.yml side_char output_folder."
              << std::endl;
    std::cout << "Attempting to run with default paramters..." << std::endl;
    in.REF_PATH = dir_of(argv[0]) + "/";
    in.FILE_STEM = "L7Y9_control1_L";
    in.CONFIG_FILE = in.REF_PATH + "config.yml";
    in.VIDEO_FILE = in.REF_PATH + "L7Y9_control1_L.avi";
    in.BKG_FILE = in.REF_PATH + "L7Y9_control1_L.png";
    in.MODEL_FILE = in.REF_PATH + "model_LocoMouse_paper.yml";
    in.CALIBRATION_FILE = in.REF_PATH + "IDX_pen_correct_fields2.yml";
    in.FLIP_CHAR = "L";
    in.OUTPUT_PATH = in.REF_PATH + ".";
    in.METHOD = "0";
  } else {
    in.VIDEO_FILE = argv[3];
    in.CONFIG_FILE = argv[2];
    in.REF_PATH = dir_of(argv[0]) + "/";
    in.FILE_STEM = strip_file_name(in.VIDEO_FILE);
    in.MODEL_FILE = argv[5];
    in.BKG_FILE = argv[4];
    in.CALIBRATION_FILE = argv[6];
    in.FLIP_CHAR = argv[7];
    in.OUTPUT_PATH = argv[8];
    in.METHOD = argv[1];
  }
  FsNode cal;
  if (!read_file_storage(in.CALIBRATION_FILE, cal))
    throw std::invalid_argument("Error: Could not open the calibration file: " + in.CALIBRATION_FILE + ".\n");
  const FsMat C = cal["ind_warp_mapping"].to_mat();
  if (C.empty()) throw std::invalid_argument("ind_warp_mapping is empty or undefined.");
  const FsMat V = cal["view_boxes"].to_mat();
  if (V.empty()) throw std::invalid_argument("view_boxes is empty or undefined.");
  if (V.rows != 2 || V.cols != 4) throw std::invalid_argument("view_boxes sould be a 2x4 matrix.");
  if (V.dt != 'i') throw std::invalid_argument("Bounding boxes must be defined with integer pixel positions!");
  if (C.dt != 'i') throw std::invalid_argument("ind_warp_mapping must be an integer (dt: i) matrix.");
  in.calib_rows = C.rows;
  in.calib_cols = C.cols;
  in.CALIBRATION.assign(C.v.begin(), C.v.end());
  in.BB_SIDE_VIEW = lm_rect{(int)V.v[0], (int)V.v[1], (int)V.v[2], (int)V.v[3]};
  in.BB_BOTTOM_VIEW = lm_rect{(int)V.v[4], (int)V.v[5], (int)V.v[6], (int)V.v[7]};
  return in;
}

// V >> F in video order; a whole batch at a time is decoded straight into
// the caller's batch buffer by worker threads (pread at each frame's offset
// in the file), so decoding is parallel and costs no extra copy.
class VideoFrames {
 public:
  VideoFrames(std::shared_ptr<AviReader> v, int threads)
      : V(std::move(v)), T(threads), FB((size_t)V->rows() * V->cols()) {}
  bool read(uint8_t* dst) { return pos < V->frame_count() && V->read_at(pos++, dst); }
  int read(uint8_t* dst, int n) {
    const auto t0 = std::chrono::steady_clock::now();
    n = (int)std::min<size_t>((size_t)std::max(n, 0), V->frame_count() - pos);
    std::vector<char> ok((size_t)n, 0);
    std::atomic<int> next{0};
    auto work = [&] {
      for (int i; (i = next++) < n;) ok[i] = V->read_at(pos + (size_t)i, dst + (size_t)i * FB) ? 1 : 0;
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < std::min(T, n); ++t) pool.emplace_back(work);
    work();
    for (auto& th : pool) th.join();
    int got = 0;
    while (got < n && ok[got]) ++got;
    pos += (size_t)got;
    decode_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return got;
  }
  int threads() const { return T; }
  double decode_s = 0;  // wall seconds in read(dst, n): file reads + decoding on T threads
  void rewind() { pos = 0; }  // V.set(CV_CAP_PROP_POS_FRAMES, 0)

 private:
  std::shared_ptr<AviReader> V;
  const int T;
  const size_t FB;
  size_t pos = 0;
};

// LocoMouse_Parameters (LocoMouse_class.cpp:4-249): keys in the reference's
// order, its messages, OpenCV's missing-key-reads-0 semantics.
struct DebugConfig {
  bool verbose = false;  // LM_DEBUG (verbose_debug, :17-19)
  int n_frames = 0;      // LM_N_FRAMES_TO_DEBUG (N_debug_frames, :21-26)
};

void load_config(const std::string& file, const std::string& ref_path, lm_params& P, lm_bb_params& B,
                 DebugConfig& D) {
  FsNode c;
  if (!read_file_storage(file, c)) throw std::invalid_argument("Failed to read config file: " + file + ".");
  const std::string E = "Invalid configuration parameter: ";
  auto bad = [&](const std::string& m) { throw std::invalid_argument(E + m); };
  auto num = [](double v) { return std::to_string(v); };
  D.verbose = c["verbose_debug"].to_int() != 0;
  D.n_frames = c["N_debug_frames"].to_int();
  if (D.n_frames < 0) bad("N_debug_frames must not be negative.");
  P.conn_comp_connectivity = c["conn_comp_connectivity"].to_int();
  if (P.conn_comp_connectivity != 4 && P.conn_comp_connectivity != 8)
    bad("conn_comp_connectivity must be either 4 or 8. Was " + std::to_string(P.conn_comp_connectivity) + ".");
  B.conn_comp_connectivity = P.conn_comp_connectivity;
  B.median_filter_size = c["median_filter_size"].to_int();
  if (B.median_filter_size % 2 == 0)
    bad("median_filter_size must be odd. Was " + std::to_string(B.median_filter_size) + ".");
  B.min_pixel_visible = c["min_pixel_visible"].to_int();
  if (B.min_pixel_visible < 0)
    bad("min_pixel_visible must be non-negative. Was " + std::to_string(B.min_pixel_visible) + ".");
  P.side_bottom_min_overlap = c["side_bottom_min_overlap"].to_double();
  if (P.side_bottom_min_overlap < 0 || P.side_bottom_min_overlap > 1)
    bad("side_bottom_min_overlap must belong to [0,1]. Was " + num(P.side_bottom_min_overlap) + ".");
  auto nonneg_int = [&](const char* key, int32_t& dst, const char* text) {
    dst = c[key].to_int();
    if (dst < 0) bad(std::string(key) + text + std::to_string(dst) + ".");
  };
  nonneg_int("max_displacement_bottom", P.max_displacement_bottom, " must be non-negative. Was ");
  nonneg_int("max_displacement_side", P.max_displacement_side, " must be non-negative. Was ");
  nonneg_int("occlusion_grid_spacing_pixels_side", P.occlusion_grid_spacing_pixels_side, " must be non-negative. Was ");
  nonneg_int("occlusion_grid_spacing_pixels_bottom", P.occlusion_grid_spacing_pixels_bottom,
             " must be non-negative.. Was ");
  P.occlusion_grid_max_width = c["occlusion_grid_max_width"].to_double();
  if (P.occlusion_grid_max_width < 0 || P.occlusion_grid_max_width > 1)
    bad("occlusion_grid_max_width must be non-negative. Was " + num(P.occlusion_grid_max_width) + ".");
  P.tail_sub_bounding_box = c["tail_sub_bounding_box"].to_double();
  if (P.tail_sub_bounding_box < 0 || P.tail_sub_bounding_box > 1)
    bad("tail_sub_bounding_box must be non-negative. Was " + num(P.tail_sub_bounding_box) + ".");
  auto nonneg = [&](const char* key, double& dst) {
    dst = c[key].to_double();
    if (dst < 0) bad(std::string(key) + " must be non-negative. Was " + num(dst) + ".");
  };
  nonneg("alpha_vel_bottom", P.alpha_vel_bottom);
  nonneg("alpha_vel_side", P.alpha_vel_side);
  nonneg("pairwise_occluded_cost", P.pairwise_occluded_cost);
  B.moving_average_window = c["moving_average_window"].to_int();
  if (B.moving_average_window % 2 == 0)
    bad("moving_average_window must be odd. Was " + std::to_string(B.moving_average_window) + ".");
  const FsMat W = c["location_prior"].to_mat();
  if (W.cols != 7 || W.rows != 5) bad("location_prior must be a 5x7 matrix. Was " + std::to_string(W.rows) + ".");
  if (W.dt != 'd') bad("location_prior must be a double (dt: d) matrix.");  // read through ptr<double>
  for (int r = 0; r < 5; ++r)
    P.location_prior[r] = lm_location_prior{W.at(r, 0), W.at(r, 1), W.at(r, 2), W.at(r, 3),
                                            W.at(r, 4), W.at(r, 5), W.at(r, 6)};
  P.transform_gray_values = c["transform_gray_values"].to_int();
  P.use_reference_image_brightness = c["use_reference_image_brightness"].to_int();
  bool both = false;
  if (P.transform_gray_values & P.use_reference_image_brightness) {
    std::cout << "Only one of 'use_reference_image_brightness' or 'transform_gray_values' should be true. Attempting "
                 "to read reference image..."
              << std::endl;
    both = true;
  }
  if (P.use_reference_image_brightness) {
    const std::string name = c["reference_image_path"].to_string();
    int r = 0, cc = 0;
    std::vector<uint8_t> px;
    if (!read_png_gray(name, r, cc, px) && !read_png_gray(ref_path + "/" + name, r, cc, px)) {
      if (both) {
        std::cout << "Could not open the reference image. Applying the provided transformation on the gray levels..."
                  << std::endl;
        P.use_reference_image_brightness = 0;
        both = false;
      } else {
        bad("Failed to open reference image: " + name + ".");
      }
    }
  }
  if (P.transform_gray_values & ~(int)both) {
    const FsMat G = c["gray_value_transformation"].to_mat();
    if (G.empty()) bad("Could not load the gray level transformation from the config file.");
    if (G.rows != 1 || G.cols != 256)
      bad("The gray level transformation must be a 1x256 matrix, was " + std::to_string(G.rows) + "x" +
          std::to_string(G.cols) + ".");
    for (int k = 0; k < 256; ++k) P.gray_value_transformation[k] = (float)G.v[k];
    // the table keeps its FileStorage depth: LUT() gives its output that type (:1448)
    static const char kDt[] = "ucwsifd";
    const char* d = std::strchr(kDt, G.dt);
    P.gray_value_transformation_depth = d ? (int32_t)(d - kDt) : LM_DEPTH_64F;
  }
  P.use_provided_bounding_box = c["use_provided_bounding_box"].to_int();
  if (P.use_provided_bounding_box) {
    const FsMat S = c["bounding_box_side"].to_mat();
    if (S.rows != 1 || S.cols != 4) {
      std::cout << S.rows << " " << S.cols << std::endl;
      bad("bounding_box_side must be a 1x4 OpenCV matrix.");
    }
    P.bounding_box_side = lm_rect{(int)S.v[0], (int)S.v[1], (int)S.v[2], (int)S.v[3]};
    const FsMat Bb = c["bounding_box_bottom"].to_mat();
    if (Bb.rows != 1 || Bb.cols != 4) bad("bounding_box_bottom must be a 1x4 OpenCV matrix.");
    if (Bb.dt != 'i')
      std::cout << "bounding_box_bottom must be provided as a 1x4 opencv matrix of type in (yml: i)." << std::endl;
    P.bounding_box_bottom = lm_rect{(int)Bb.v[0], (int)Bb.v[1], (int)Bb.v[2], (int)Bb.v[3]};
  }
}

struct Model {  // LocoMouse_Model (:3095-3162)
  std::vector<double> w[6];
  lm_model m{};
};

void load_model(const std::string& file, Model& M) {
  FsNode c;
  if (!read_file_storage(file, c)) throw std::invalid_argument("Error: Could not open the model file: " + file + "\n");
  static const char* names[6] = {"modelPaw_side", "modelPaw_bottom", "modelTail_side",
                                 "modelTail_bottom", "modelSnout_side", "modelSnout_bottom"};
  static const char* biases[6] = {"biasPaw_side", "biasPaw_bottom", "biasTail_side",
                                  "biasTail_bottom", "biasSnout_side", "biasSnout_bottom"};
  lm_detector* dst[6] = {&M.m.paw_side, &M.m.paw_bottom, &M.m.tail_side,
                         &M.m.tail_bottom, &M.m.snout_side, &M.m.snout_bottom};
  for (int k = 0; k < 6; ++k) {
    const FsMat W = c[names[k]].to_mat();
    if (W.empty()) throw std::invalid_argument(std::string("Error: ") + names[k] + " cannot be empty." + file + "\n");
    M.w[k] = W.v;
    dst[k]->rows = W.rows;
    dst[k]->cols = W.cols;
  }
  for (int k = 0; k < 6; ++k) {
    dst[k]->weights = M.w[k].data();
    dst[k]->bias = c[biases[k]].to_double();
  }
}

int run(int argc, char** argv) {
  ParsedInputs in = parse_inputs(argc, argv);
  LocoMouse_Inputs li;
  const int method = std::stoi(in.METHOD);  // LocoMouse::initializePaths
  DebugConfig dbg;
  load_config(in.CONFIG_FILE, in.REF_PATH, li.params, li.bb_params, dbg);
  auto video = std::make_shared<AviReader>();
  if (!video->open(in.VIDEO_FILE)) throw std::invalid_argument("Could not open the video file: " + in.VIDEO_FILE + ".");
  li.n_frames = video->frame_count();
  if (dbg.verbose && dbg.n_frames > 0)  // loadVideo (:380-389): debugging runs the first N_debug_frames only
    li.n_frames = std::min<uint32_t>(li.n_frames, (uint32_t)dbg.n_frames);
  li.verbose_debug = dbg.verbose;
  li.debug_file = in.OUTPUT_PATH + "/debug_" + in.FILE_STEM + ".yml";  // initializePaths (:361-362)
  li.debug_text = in.OUTPUT_PATH + "/debug_" + in.FILE_STEM + ".txt";
  if (li.n_frames < 1) throw std::invalid_argument("Error: Video has no images to read from.");
  int br = 0, bc = 0;
  std::vector<uint8_t> bkg;
  if (!read_png_gray(in.BKG_FILE, br, bc, bkg))
    throw std::invalid_argument("Could not open the background image: " + in.BKG_FILE + ".");
  if (bc != video->cols() || br != video->rows()) {  // validateImageVideoSize (:486-492)
    std::ostringstream m;
    m << "Error: Background image does not match video size. Background image has size [" << bc << " x " << br
      << "] while Video has size [" << video->cols() << " x " << video->rows() << "]." << '\n';
    throw std::runtime_error(m.str());
  }
  Model model;
  load_model(in.MODEL_FILE, model);
  if (in.FLIP_CHAR.size() != 1 || (in.FLIP_CHAR[0] != 'L' && in.FLIP_CHAR[0] != 'R'))
    throw std::invalid_argument("Mouse side option must be either \"L\" or \"R\".");
  li.setup.method = method;
  li.setup.flip = in.FLIP_CHAR[0] == 'L';
  li.setup.video_rows = video->rows();
  li.setup.video_cols = video->cols();
  li.setup.background = bkg.data();
  li.setup.calib_rows = in.calib_rows;
  li.setup.calib_cols = in.calib_cols;
  li.setup.ind_warp_mapping = in.CALIBRATION.data();
  li.setup.view_box_side = in.BB_SIDE_VIEW;
  li.setup.view_box_bottom = in.BB_BOTTOM_VIEW;
  li.model = model.m;
  // Decode threads: MJPEG frames decode at a few hundred per second per core,
  // so a batch is spread over up to 16 (LM_READ_THREADS overrides).
  int read_threads = std::max(1, std::min(16, (int)std::thread::hardware_concurrency()));
  if (const char* t = std::getenv("LM_READ_THREADS")) read_threads = std::max(1, std::atoi(t));
  auto reader = std::make_shared<VideoFrames>(video, read_threads);
  li.read_frame = [reader](uint8_t* dst) { return reader->read(dst); };
  li.read_frames = [reader](uint8_t* dst, int n) { return reader->read(dst, n); };
  li.rewind = [reader] { reader->rewind(); };
  li.output_file = in.OUTPUT_PATH + "/output_" + in.FILE_STEM + ".yml";
  if (const char* d = std::getenv("LM_DEVICE")) li.device = std::atoi(d);
  // LM_DEVICES=0,1,...: detection sharded over these GPUs (LocoMouse_Inputs::devices);
  // LM_OVERSUBSCRIBE=1 lets a device appear more than once (rehearsals on fewer GPUs)
  if (const char* ds = std::getenv("LM_DEVICES")) {
    std::stringstream ss(ds);
    std::string tok;
    while (std::getline(ss, tok, ','))
      if (!tok.empty()) {
        size_t used = 0;
        int d = -1;
        try {
          d = std::stoi(tok, &used);
        } catch (const std::exception&) {
          used = 0;
        }
        if (used != tok.size()) throw std::invalid_argument("LM_DEVICES: not a device index: " + tok);
        li.devices.push_back(d);
      }
  }
  if (const char* o = std::getenv("LM_OVERSUBSCRIBE")) li.oversubscribe = std::atoi(o) != 0;
  if (const char* b = std::getenv("LM_BATCH")) li.batch = std::max(1, std::atoi(b));
  if (const char* l = std::getenv("LM_LANES")) li.lanes = std::max(1, std::atoi(l));
  if (std::getenv("LM_PRINT_INPUTS")) {  // diagnostics: the parsed inputs, nothing run on the GPU
    const lm_params& P = li.params;
    std::cout << "method " << method << "\nflip " << li.setup.flip << "\nvideo " << li.setup.video_rows << " "
              << li.setup.video_cols << " " << li.n_frames << "\ncalib " << in.calib_rows << " " << in.calib_cols
              << "\noutput " << li.output_file << "\nconn " << P.conn_comp_connectivity << "\nmax_disp "
              << P.max_displacement_bottom << " " << P.max_displacement_side << "\nong_spacing "
              << P.occlusion_grid_spacing_pixels_side << " " << P.occlusion_grid_spacing_pixels_bottom
              << "\nuse_bb " << P.use_provided_bounding_box << "\nbb_side " << P.bounding_box_side.x << " "
              << P.bounding_box_side.y << " " << P.bounding_box_side.width << " " << P.bounding_box_side.height
              << "\nbb_bottom " << P.bounding_box_bottom.x << " " << P.bounding_box_bottom.y << " "
              << P.bounding_box_bottom.width << " " << P.bounding_box_bottom.height << "\nbb_params "
              << li.bb_params.median_filter_size << " " << li.bb_params.min_pixel_visible << " "
              << li.bb_params.moving_average_window << "\n";
    std::cout.precision(17);
    std::cout << "doubles " << P.side_bottom_min_overlap << " " << P.occlusion_grid_max_width << " "
              << P.tail_sub_bounding_box << " " << P.alpha_vel_bottom << " " << P.alpha_vel_side << " "
              << P.pairwise_occluded_cost << "\nprior";
    for (int r = 0; r < 5; ++r)
      for (double v : {P.location_prior[r].x, P.location_prior[r].y, P.location_prior[r].max_distance,
                       P.location_prior[r].min_x, P.location_prior[r].max_x, P.location_prior[r].min_y,
                       P.location_prior[r].max_y})
        std::cout << " " << v;
    const lm_detector* dets[6] = {&li.model.paw_bottom, &li.model.paw_side, &li.model.snout_bottom,
                                  &li.model.snout_side, &li.model.tail_bottom, &li.model.tail_side};
    for (const lm_detector* d : dets) {
      double sum = 0;
      for (int k = 0; k < d->rows * d->cols; ++k) sum += d->weights[k];
      std::cout << "\ndetector " << d->rows << " " << d->cols << " " << d->bias << " " << sum;
    }
    unsigned long long bsum = 0;
    for (uint8_t v : bkg) bsum += v;
    std::cout << "\nbackground_sum " << bsum << std::endl;
    return EXIT_SUCCESS;
  }
  {  // OUTPUT = FileStorage(output_file, WRITE) must open (:333-337)
    std::FILE* f = std::fopen(li.output_file.c_str(), "w");
    if (!f) throw std::runtime_error("Could not create output file:  " + li.output_file + "\n");
    std::fclose(f);
  }

  const auto t_start = std::chrono::steady_clock::now();
  std::unique_ptr<LocoMouse> L = LocoMouse_Initialize(li);  // main.cpp:45-91
  L->getBoundingBox();
  L->initializeFeatureLoop();
  const auto t_init = std::chrono::steady_clock::now();
  const double decode_init = reader->decode_s;  // the bounding-box pass's reads, when it runs
  for (unsigned int i = 0; i < L->N_frames(); ++i) {
    L->readFrame();
    L->cropBoundingBox();
    L->detectTail();
    L->detectBottomCandidates();
    L->computeUnaryCostsBottom();
    L->computePairwiseCostsBottom();
    L->detectSideCandidates();
    L->matchBottomSideCandidates();
    L->storePreviousImage();
  }
  const auto t_loop = std::chrono::steady_clock::now();
  L->computeBottomTracks();
  L->computeSideTracks();
  const auto t_tracks = std::chrono::steady_clock::now();
  L->exportResults();
  if (std::getenv("LM_TIMING")) {  // stage times (not in the reference)
    const auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    const LocoMouse::StageTimes st = L->stage_times();
    std::cout << "LM_TIMING init_ms " << ms(t_start, t_init) << " loop_ms " << ms(t_init, t_loop) << " tracks_ms "
              << ms(t_loop, t_tracks) << " export_ms " << ms(t_tracks, std::chrono::steady_clock::now())
              << " decode_ms " << 1e3 * (reader->decode_s - decode_init) << " decode_threads " << reader->threads()
              << " submit_ms " << 1e3 * st.submit_s << " wait_ms " << 1e3 * st.wait_s << " batches " << st.batches
              << " frames " << L->N_frames() << std::endl;
  }
  return EXIT_SUCCESS;
}

}  // namespace
}  // namespace locomouse

int main(int argc, char* argv[]) {
  const auto t0 = std::chrono::steady_clock::now();
  int return_val = EXIT_SUCCESS;
  try {
    return_val = locomouse::run(argc, argv);
  } catch (const std::invalid_argument& e) {
    std::cout << "Invalid inputs: " << e.what() << std::endl;
    return_val = EXIT_FAILURE;
  } catch (const std::runtime_error& e) {
    std::cout << "Runtime Error: " << e.what() << std::endl;
    return_val = EXIT_FAILURE;
  }
  const double t = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  std::cout << "Total Elapsed time: " << t << "s" << std::endl;
  return return_val;
}
