// gol_frontend.cpp -- native host-side mirror of the reference's frontend
// (Run.scala RunFrontend, BoardCreator.scala, LoggerActor.scala) driving the
// GPU generation step through the C ABI only (include/gol.h; built with g++,
// no HIP headers).
//
//   gol_frontend [--config FILE] [--quiet] [key=value ...]
//
// Config keys are the reference's (application.conf:29-47) plus the build's
// (SURVEY.md section 5):
//   game-of-life.board.size.x / .y            board size (w, h): (w+1) x (h+1) cells
//   game-of-life.board.topology               ref-clipped (default) | torus
//   game-of-life.simulation.rule              ref-effective (default) | ref-literal | life | B../S..
//   game-of-life.simulation.seed              java.util.Random seed (ref-clipped) / splitmix64 seed (torus)
//   game-of-life.simulation.generations       NextStep ticks to run (default 100)
//   game-of-life.simulation.tick              pause between ticks (default 0ms here; the reference: 3000ms)
//   game-of-life.simulation.gpus              devices to spread row-block shards over (default 1)
//   game-of-life.simulation.shards            shards (default = gpus); > 1 runs an in-process group
//   game-of-life.log.file                     LoggerActor output (default info.log, "-" = stdout)
//   game-of-life.log.every                    log the board every N epochs (0 = never; default 1)
//   game-of-life.log.full                     false (default): the reference's dump shape; true: the
//                                             whole board (this build's extension)
//
// Output: "Epoch: N" per tick on stdout (BoardCreator.scala:115) unless
// --quiet, "hash N 0x<16 hex>" per generation, and the LoggerActor board
// dump in the reference's shape for board size (x, y): "At epoch:N", 2x+1
// dashes, y rows "[a,b,...]" of x entries, the dashes again and an empty line
// (LoggerActor.scala:17,28,36-44) -- the cells of columns 0..x-1 and rows
// 0..y-1, positional here (the reference prints x*y of the (x+1)*(y+1) cells
// in arrival order).  log.full=true prints every row and column instead.
#include <chrono>
#include <cinttypes>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <map>
#include <regex>
#include <sstream>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../../include/gol.h"

namespace {

using Config = std::map<std::string, std::string>;

void check(int rc, const gol_ctx* ctx, const char* what) {
    if (rc != GOL_OK) {
        throw std::runtime_error(std::string(what) + ": " + gol_strerror(rc) + ": " + gol_last_error(ctx));
    }
}

// Minimal HOCON reader (nested blocks, key = value, // and # comments),
// flattened to dotted keys -- enough for application.conf.
void parse_hocon(const std::string& text, Config& out) {
    std::vector<std::string> stack;
    std::istringstream in(text);
    std::string line;
    const std::regex kv(R"(^\s*([\w.\-"]+)\s*[=:]\s*(.+?)\s*$)");
    while (std::getline(in, line)) {
        const size_t c1 = line.find("//"), c2 = line.find('#');
        line = line.substr(0, std::min(c1, c2));
        const size_t a = line.find_first_not_of(" \t\r"), b = line.find_last_not_of(" \t\r");
        if (a == std::string::npos) continue;
        line = line.substr(a, b - a + 1);
        if (line.back() == '{') {
            std::string key = line.substr(0, line.size() - 1);
            key.erase(key.find_last_not_of(" \t") + 1);
            stack.push_back(key);
            continue;
        }
        if (line == "}") {
            if (!stack.empty()) stack.pop_back();
            continue;
        }
        std::smatch m;
        if (std::regex_match(line, m, kv)) {
            std::string key;
            for (const auto& s : stack) key += s + ".";
            std::string k = m[1].str(), v = m[2].str();
            if (!k.empty() && k.front() == '"') k = k.substr(1, k.size() - 2);
            if (!v.empty() && v.front() == '"') v = v.substr(1, v.size() - 2);
            out[key + k] = v;
        }
    }
}

int64_t duration_ms(const std::string& v) {
    std::smatch m;
    if (!std::regex_match(v, m, std::regex(R"(\s*(\d+)\s*([a-z]*)\s*)"))) throw std::runtime_error("bad duration " + v);
    const int64_t n = std::stoll(m[1].str());
    const std::string u = m[2].str();
    if (u.empty() || u == "ms" || u == "millis" || u == "millisecond" || u == "milliseconds") return n;
    if (u == "s" || u == "second" || u == "seconds") return n * 1000;
    if (u == "m" || u == "minute" || u == "minutes") return n * 60000;
    throw std::runtime_error("bad duration unit " + u);
}

void parse_rule(const std::string& name, uint32_t& birth, uint32_t& survive) {
    if (name == "life") { birth = GOL_RULE_LIFE_BIRTH; survive = GOL_RULE_LIFE_SURVIVE; return; }
    if (name == "ref-literal") { birth = GOL_RULE_REF_LITERAL_BIRTH; survive = GOL_RULE_REF_LITERAL_SURVIVE; return; }
    if (name == "ref-effective") {
        birth = GOL_RULE_REF_EFFECTIVE_BIRTH; survive = GOL_RULE_REF_EFFECTIVE_SURVIVE; return;
    }
    std::smatch m;
    if (!std::regex_match(name, m, std::regex(R"([Bb]([0-8]*)/[Ss]([0-8]*))"))) throw std::runtime_error("bad rule " + name);
    birth = survive = 0;
    for (char c : m[1].str()) birth |= 1u << (c - '0');
    for (char c : m[2].str()) survive |= 1u << (c - '0');
}

// BoardCreator.scala:23 with a seeded java.util.Random: the k-th
// nextBoolean() goes to the k-th position of generateAllCoordinates
// (BoardCreator.scala:47-53: i in 0..w outer, j in 0..h inner).
std::vector<uint8_t> java_random_board(int w, int h, int64_t seed) {
    const uint64_t mult = 0x5DEECE66DULL, add = 0xBULL, mask = (1ULL << 48) - 1;
    uint64_t s = ((uint64_t)seed ^ mult) & mask;
    std::vector<uint8_t> cells((size_t)(w + 1) * (h + 1));
    for (int i = 0; i <= w; ++i)
        for (int j = 0; j <= h; ++j) {
            s = (s * mult + add) & mask;
            cells[(size_t)j * (w + 1) + i] = (uint8_t)((s >> 47) != 0);  // next(1) != 0
        }
    return cells;
}

// LoggerActor.scala:17-19,36-44 text format: `x` entries per row, `y` rows.
class LoggerActor {
  public:
    LoggerActor(int x, int y, const std::string& path) : x_(x), y_(y) {
        if (path != "-") {
            file_.open(path, std::ios::app);  // logback.xml: FileAppender, append
            if (!file_) throw std::runtime_error("cannot open log file " + path);
            out_ = &file_;
        }
    }
    void log_board(const std::vector<uint32_t>& packed, int64_t words_per_row, uint64_t epoch) {
        std::ostream& o = *out_;
        const std::string dash(2 * x_ + 1, '-');
        o << "At epoch:" << epoch << "\n" << dash << "\n";
        for (int r = 0; r < y_; ++r) {
            o << "[";
            for (int c = 0; c < x_; ++c)
                o << (c ? "," : "") << ((packed[(size_t)r * words_per_row + c / 32] >> (c % 32)) & 1u);
            o << "]\n";
        }
        o << dash << "\n\n";
        o.flush();
    }

  private:
    int x_, y_;
    std::ofstream file_;
    std::ostream* out_ = &std::cout;
};

// BoardCreator (BoardCreator.scala:18-155) over GPU shard contexts.
class BoardCreator {
  public:
    BoardCreator(const Config& cfg) {
        x_ = std::stoi(cfg.at("game-of-life.board.size.x"));
        y_ = std::stoi(cfg.at("game-of-life.board.size.y"));
        torus_ = cfg.at("game-of-life.board.topology") == "torus";
        parse_rule(cfg.at("game-of-life.simulation.rule"), birth_, survive_);
        seed_ = std::stoll(cfg.at("game-of-life.simulation.seed"), nullptr, 0);
        tick_ms_ = duration_ms(cfg.at("game-of-life.simulation.tick"));
        const int gpus = std::max(1, std::stoi(cfg.at("game-of-life.simulation.gpus")));
        const int shards = std::max(1, std::stoi(cfg.at("game-of-life.simulation.shards")));
        // ref-clipped: (w+1) x (h+1) cells, neighbours in [0,w) x [0,h);
        // torus: a w x h ring (w multiple of 32)
        width_ = torus_ ? x_ : x_ + 1;
        height_ = torus_ ? y_ : y_ + 1;
        for (int k = 0; k < shards; ++k) {
            int64_t row0 = 0, rows = 0;
            check(gol_shard_rows(height_, k, shards, &row0, &rows), nullptr, "gol_shard_rows");
            gol_config c{};
            c.width = width_;
            c.height = height_;
            c.row0 = row0;
            c.rows = rows;
            c.topology = torus_ ? GOL_TORUS : GOL_REF_CLIPPED;
            c.birth_mask = birth_;
            c.survive_mask = survive_;
            c.device = k % gpus;
            gol_ctx* ctx = nullptr;
            check(gol_create(&ctx, &c), nullptr, "gol_create");
            ctxs_.push_back(ctx);
            row0s_.push_back(row0);
            rows_.push_back(rows);
        }
        initial_state();
        if (ctxs_.size() > 1) {
            if (gol_group_create(&group_, ctxs_.data(), (int)ctxs_.size()) != GOL_OK)
                throw std::runtime_error(std::string("gol_group_create: ") + gol_last_error(nullptr));
        }
    }
    ~BoardCreator() {
        if (group_) gol_group_destroy(group_);
        for (gol_ctx* c : ctxs_) gol_destroy(c);
    }

    void start_simulation() { running_ = true; }   // :105-108
    void pause_simulation() { running_ = false; }  // :109-110
    void resume_simulation() { running_ = true; }  // :111-112

    // :113-116 NextStep: step += 1, CurrentEpochMsg(step) to every cell
    uint64_t next_step() {
        if (!running_) return 0;
        step_ += 1;
        uint64_t h = 0;
        if (group_) {
            if (gol_group_step(group_, 1, &h) != GOL_OK)
                throw std::runtime_error(std::string("gol_group_step: ") + gol_group_last_error(group_));
        } else {
            check(gol_step(ctxs_[0], 1, &h), ctxs_[0], "gol_step");
        }
        return h;
    }

    std::vector<uint32_t> snapshot() const {
        const int64_t wpr = (width_ + 31) / 32;
        std::vector<uint32_t> out((size_t)height_ * wpr);
        for (size_t k = 0; k < ctxs_.size(); ++k)
            check(gol_snapshot(ctxs_[k], out.data() + row0s_[k] * wpr, wpr), ctxs_[k], "gol_snapshot");
        return out;
    }

    int64_t tick_ms() const { return tick_ms_; }
    int64_t words_per_row() const { return (width_ + 31) / 32; }
    int x() const { return torus_ ? x_ : x_ + 1; }  // cells per row
    int y() const { return torus_ ? y_ : y_ + 1; }  // rows
    int size_x() const { return x_; }               // board size (x, y) (application.conf:31-33)
    int size_y() const { return y_; }
    uint64_t step() const { return step_; }

  private:
    void initial_state() {
        const int64_t wpr = (width_ + 31) / 32;
        if (torus_) {
            for (gol_ctx* c : ctxs_) check(gol_seed(c, (uint64_t)seed_), c, "gol_seed");
            return;
        }
        const std::vector<uint8_t> cells = java_random_board(x_, y_, seed_);
        std::vector<uint32_t> packed((size_t)height_ * wpr, 0u);
        for (int64_t r = 0; r < height_; ++r)
            for (int64_t c = 0; c < width_; ++c)
                if (cells[(size_t)r * width_ + c]) packed[(size_t)r * wpr + c / 32] |= 1u << (c % 32);
        for (size_t k = 0; k < ctxs_.size(); ++k)
            check(gol_load(ctxs_[k], packed.data() + row0s_[k] * wpr, wpr), ctxs_[k], "gol_load");
    }

    int x_ = 6, y_ = 6;
    bool torus_ = false;
    uint32_t birth_ = 0, survive_ = 0x1FF;
    int64_t seed_ = 0, tick_ms_ = 0, width_ = 0, height_ = 0;
    std::vector<gol_ctx*> ctxs_;
    std::vector<int64_t> row0s_, rows_;
    gol_group* group_ = nullptr;
    bool running_ = false;
    uint64_t step_ = 0;
};

}  // namespace

int main(int argc, char** argv) {
    Config cfg = {
        {"game-of-life.board.size.x", "6"},            // application.conf:32
        {"game-of-life.board.size.y", "6"},            // application.conf:33
        {"game-of-life.simulation.tick", "0ms"},       // reference default 3000ms (:40)
        {"game-of-life.simulation.max-crashes", "100"},  // :41 (fault injection: gameoflife.fault)
        {"game-of-life.board.topology", "ref-clipped"},
        {"game-of-life.simulation.rule", "ref-effective"},
        {"game-of-life.simulation.seed", "42"},
        {"game-of-life.simulation.generations", "100"},
        {"game-of-life.simulation.gpus", "1"},
        {"game-of-life.log.file", "info.log"},
        {"game-of-life.log.every", "1"},
        {"game-of-life.log.full", "false"},
    };
    bool quiet = false;
    try {
        if (gol_abi_version() != GOL_ABI_VERSION)
            throw std::runtime_error("libgol ABI version " + std::to_string(gol_abi_version()) +
                                     ", this frontend was built against " + std::to_string(GOL_ABI_VERSION));
        for (int i = 1; i < argc; ++i) {
            std::string a = argv[i];
            if (a == "--quiet") { quiet = true; continue; }
            if (a == "--config" && i + 1 < argc) {
                std::ifstream f(argv[++i]);
                if (!f) throw std::runtime_error(std::string("cannot read ") + argv[i]);
                std::stringstream ss;
                ss << f.rdbuf();
                parse_hocon(ss.str(), cfg);
                continue;
            }
            const size_t eq = a.find('=');
            if (eq == std::string::npos) throw std::runtime_error("expected key=value, got " + a);
            std::string k = a.substr(0, eq);
            if (k.rfind("game-of-life.", 0) != 0) k = "game-of-life." + k;
            cfg[k] = a.substr(eq + 1);
        }
        if (!cfg.count("game-of-life.simulation.shards"))
            cfg["game-of-life.simulation.shards"] = cfg["game-of-life.simulation.gpus"];
        BoardCreator board(cfg);
        // the reference's LoggerActor(boardSize): x*y cells per epoch
        // (LoggerActor.scala:28); log.full: the whole board
        const bool full = cfg["game-of-life.log.full"] == "true";
        LoggerActor logger(full ? board.x() : board.size_x(), full ? board.y() : board.size_y(),
                           cfg["game-of-life.log.file"]);
        const int64_t gens = std::stoll(cfg["game-of-life.simulation.generations"]);
        const int64_t every = std::stoll(cfg["game-of-life.log.every"]);
        board.start_simulation();
        for (int64_t g = 0; g < gens; ++g) {
            const uint64_t h = board.next_step();
            if (!quiet) std::printf("Epoch: %" PRIu64 "\n", board.step());
            std::printf("hash %" PRIu64 " 0x%016" PRIx64 "\n", board.step(), h);
            if (every > 0 && board.step() % (uint64_t)every == 0)
                logger.log_board(board.snapshot(), board.words_per_row(), board.step());
            if (board.tick_ms() > 0) std::this_thread::sleep_for(std::chrono::milliseconds(board.tick_ms()));
        }
    } catch (const std::exception& e) {
        std::fprintf(stderr, "gol_frontend: %s\n", e.what());
        return 1;
    }
    return 0;
}
