// El::Gemm experiment-suite driver over the drop-in header (include/El.hpp):
// takes the reference suite's experiment files unchanged
// (tests/blas_like/Gemm_Suite.cpp:274-276: one experiment per line,
// DEVICE:TYPE:ORIENT:ORIENT:ALG:M:N:K:BLK_SIZE, lines that do not match are
// skipped as in its regex scan, :494-540) and writes the same results file
// (DEV:TYPE:ORA:ORB:ALG:M:N:K:NB:t_1:...:t_R, :617-662).  Per experiment, as the
// suite does (:137-248): Blocksize(NB), A, B, COrig = Uniform(center -0.1,
// radius 0.1), alpha = 0.5, beta = -0.5; warm-up runs C = COrig; Gemm; the
// associativity check || (alpha op(A) op(B) + beta COrig) X - C X ||_F / ||Y||_F
// with X Uniform(center -0.25, radius 0.25), 100 columns (:91-132); then timed
// runs, each preceded by untimed ones.  Types: D double, F float, H half
// (gpu_half_type), B bfloat16 (new).  One process, Grid 1x1.
//
// Inputs: --fill mt19937 draws A, B, COrig exactly as the reference does
// (El::Uniform: one host std::mt19937 stream, then a host-to-device copy: ~10 s
// per 32768^2 matrix); the default --fill hash draws the same distribution from
// the grid-independent counter hash on the device (El::HashFill), seeds 1, 2, 3.
//
// Timing: the device is synchronized around each timed Gemm and the host clock
// read (the suite reads a hipEvent pair on C's stream; both bracket exactly the
// one call).  --check makes a warm-up residual above the type's bound fatal
// (the suite only prints it).
//
//   gemm_suite --f experiments.txt --o results.txt [--warmup 5] [--runs 10]
//              [--skips 2] [--check] [--fill hash|mt19937]
#include <El.hpp>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

namespace {

struct Experiment {
    El::Device dev;
    char type;  // 'D', 'F', 'H', 'B'
    El::Orientation oa, ob;
    El::GemmAlgorithm alg;
    std::string alg_name;
    El::Int m, n, k, nb;
};

struct Options {
    std::string in, out;
    int warmup = 5, runs = 10, skips = 2;
    bool check = false;
    bool mt19937 = false;
};

const char* kAlgNames[] = {"DEFAULT", "SUMMA_A_MS", "SUMMA_A", "SUMMA_B_MS", "SUMMA_B",
                           "SUMMA_C_MS", "SUMMA_C", "SUMMA_DOT", "CANNON"};

bool ParseAlg(const std::string& s, El::GemmAlgorithm& a) {
    for (int i = 0; i < 9; ++i)
        if (s == kAlgNames[i]) {
            a = static_cast<El::GemmAlgorithm>(i);  // ordinals of level3.hpp:22-35
            return true;
        }
    return false;
}

bool ParseOrient(const std::string& s, El::Orientation& o) {
    if (s.empty()) return false;
    switch (s[0]) {  // first letter, as CharToOrientation
    case 'N': o = El::NORMAL; return true;
    case 'T': o = El::TRANSPOSE; return true;
    case 'C': case 'A': o = El::ADJOINT; return true;
    default: return false;
    }
}

bool AllAlnum(const std::string& s) {
    if (s.empty()) return false;
    for (char c : s)
        if (!std::isalnum(static_cast<unsigned char>(c))) return false;
    return true;
}

// One experiment from a line: nine ':'-separated fields, letters for the first
// four, [A-Z_] for the algorithm, alphanumerics (decimal sizes) for the rest.
bool ParseLine(const std::string& line, Experiment& e) {
    std::vector<std::string> f;
    std::stringstream ss(line);
    std::string tok;
    while (std::getline(ss, tok, ':')) f.push_back(tok);
    if (f.size() < 9) return false;
    auto trim = [](std::string s) {
        while (!s.empty() && std::isspace(static_cast<unsigned char>(s.back()))) s.pop_back();
        while (!s.empty() && std::isspace(static_cast<unsigned char>(s.front()))) s.erase(s.begin());
        return s;
    };
    for (auto& x : f) x = trim(x);
    for (int i = 0; i < 4; ++i)
        for (char c : f[i])
            if (!std::isalpha(static_cast<unsigned char>(c))) return false;
    for (int i = 5; i < 9; ++i)
        if (!AllAlnum(f[i])) return false;
    if (f[0].empty() || (f[0][0] != 'C' && f[0][0] != 'G')) return false;
    e.dev = f[0][0] == 'G' ? El::Device::GPU : El::Device::CPU;
    e.type = f[1].empty() ? '?' : f[1][0];
    if (!ParseOrient(f[2], e.oa) || !ParseOrient(f[3], e.ob)) return false;
    if (!ParseAlg(f[4], e.alg)) return false;
    e.alg_name = f[4];
    e.m = std::stoll(f[5]);
    e.n = std::stoll(f[6]);
    e.k = std::stoll(f[7]);
    e.nb = std::stoll(f[8]);
    return true;
}

const char* OrientName(El::Orientation o) {
    return o == El::NORMAL ? "Normal" : o == El::TRANSPOSE ? "Transpose" : "Adjoint";
}
const char* TypeName(char t) {
    return t == 'D' ? "double" : t == 'F' ? "float" : t == 'H' ? "half" : "bfloat16";
}

template <typename T> double Bound();  // warm-up residual bound for --check
template <> double Bound<double>() { return 1e-10; }
template <> double Bound<float>() { return 1e-3; }
template <> double Bound<El::gpu_half_type>() { return 5e-2; }
template <> double Bound<El::bfloat16>() { return 2e-1; }

template <typename T, El::Device D>
using DM = El::DistMatrix<T, El::MC, El::MR, El::ELEMENT, D>;

// || (alpha op(A) op(B) + beta COrig) X - CFinal X ||_F / || Y ||_F
template <typename T, El::Device D>
double Associativity(const Experiment& e, T alpha, const DM<T, D>& A, const DM<T, D>& B, T beta,
                     const DM<T, D>& COrig, const DM<T, D>& CFinal) {
    El::InitializeRandom();  // the same X every time
    const El::Grid& g = A.Grid();
    DM<T, D> X(g), Y(g), Z(g);
    El::Uniform(X, e.n, 100, El::detail::FromDouble<T>(-0.25), 0.25);
    const T one = El::detail::FromDouble<T>(1.0), neg = El::detail::FromDouble<T>(-1.0);
    El::Gemm(e.ob, El::NORMAL, one, B, X, Z);
    El::Gemm(e.oa, El::NORMAL, alpha, A, Z, Y);
    El::Gemm(El::NORMAL, El::NORMAL, beta, COrig, X, one, Y);
    const double ynorm = El::FrobeniusNorm(Y);
    El::Gemm(El::NORMAL, El::NORMAL, neg, CFinal, X, one, Y);
    return El::FrobeniusNorm(Y) / ynorm;
}

template <typename T, El::Device D>
std::vector<double> Run(const Experiment& e, const Options& o, const El::Grid& g, bool& ok) {
    std::printf("Testing Gemm%c%c_%s with %s on %s\n  M=%lld N=%lld K=%lld NB=%lld\n",
                OrientName(e.oa)[0], OrientName(e.ob)[0], e.alg_name.c_str(), TypeName(e.type),
                e.dev == El::Device::GPU ? "GPU" : "CPU", (long long)e.m, (long long)e.n, (long long)e.k,
                (long long)e.nb);
    El::SetBlocksize(e.nb);
    const T alpha = El::detail::FromDouble<T>(0.5), beta = El::detail::FromDouble<T>(-0.5);
    const El::Int ar = e.oa == El::NORMAL ? e.m : e.k, ac = e.oa == El::NORMAL ? e.k : e.m;
    const El::Int br = e.ob == El::NORMAL ? e.k : e.n, bc = e.ob == El::NORMAL ? e.n : e.k;
    DM<T, D> A(g), B(g), COrig(g), C(g);
    const T c0 = El::detail::FromDouble<T>(-0.1);
    if (o.mt19937) {
        El::Uniform(A, ar, ac, c0, 0.1);
        El::Uniform(B, br, bc, c0, 0.1);
        El::Uniform(COrig, e.m, e.n, c0, 0.1);
    } else {
        A.Resize(ar, ac);
        B.Resize(br, bc);
        COrig.Resize(e.m, e.n);
        El::HashFill(A, 1, -0.1, 0.1);
        El::HashFill(B, 2, -0.1, 0.1);
        El::HashFill(COrig, 3, -0.1, 0.1);
    }
    std::printf("  Correctness tests:\n");
    for (int i = 0; i < o.warmup; ++i) {
        C = COrig;
        El::Gemm(e.oa, e.ob, alpha, A, B, beta, C, e.alg);
        const double r = Associativity<T, D>(e, alpha, A, B, beta, COrig, C);
        std::printf("    || E ||_F / || Y ||_F = %.6e\n", r);
        if (o.check && !(r <= Bound<T>())) {
            std::fprintf(stderr, "associativity residual %.3e above %.1e\n", r, Bound<T>());
            ok = false;
        }
    }
    C = COrig;
    elx_device_synchronize();
    std::vector<double> times;
    for (int i = 0; i < o.runs; ++i) {
        for (int s = 0; s < o.skips; ++s) El::Gemm(e.oa, e.ob, alpha, A, B, beta, C, e.alg);
        elx_device_synchronize();
        const auto t0 = std::chrono::steady_clock::now();
        El::Gemm(e.oa, e.ob, alpha, A, B, beta, C, e.alg);
        elx_device_synchronize();
        times.push_back(std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
    }
    double mean = 0, var = 0;
    for (double t : times) mean += t;
    mean /= times.size();
    for (double t : times) var += (t - mean) * (t - mean) / std::max<size_t>(times.size() - 1, 1);
    std::printf("  Mean: %.6es, StdDev: %.6e  (%.2f GFLOP/s)\nFinished.\n\n", mean, std::sqrt(var),
                2.0 * e.m * e.n * e.k / mean / 1e9);
    return times;
}

template <El::Device D>
std::vector<double> Dispatch(const Experiment& e, const Options& o, const El::Grid& g, bool& ok) {
    switch (e.type) {
    case 'D': return Run<double, D>(e, o, g, ok);
    case 'F': return Run<float, D>(e, o, g, ok);
    case 'H': return Run<El::gpu_half_type, D>(e, o, g, ok);
    case 'B': return Run<El::bfloat16, D>(e, o, g, ok);
    default: throw El::RuntimeError("Invalid type detected.");
    }
}

}  // namespace

int main(int argc, char** argv) {
    Options o;
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        auto next = [&]() -> std::string {
            if (i + 1 >= argc) throw std::runtime_error("missing value for " + a);
            return argv[++i];
        };
        if (a == "--f") o.in = next();
        else if (a == "--o") o.out = next();
        else if (a == "--warmup") o.warmup = std::atoi(next().c_str());
        else if (a == "--runs") o.runs = std::atoi(next().c_str());
        else if (a == "--skips") o.skips = std::atoi(next().c_str());
        else if (a == "--gridHeight") next();  // one process: the grid is 1x1
        else if (a == "--check") o.check = true;
        else if (a == "--fill") {
            const std::string f = next();
            if (f != "hash" && f != "mt19937") {
                std::fprintf(stderr, "--fill hash|mt19937\n");
                return 2;
            }
            o.mt19937 = f == "mt19937";
        }
        else {
            std::fprintf(stderr, "unknown option %s\n", a.c_str());
            return 2;
        }
    }
    std::setvbuf(stdout, nullptr, _IOLBF, 0);  // progress lines as they happen
    El::Initialize(argc, argv);
    std::vector<Experiment> suite;
    {
        std::ifstream in(o.in);
        if (!in) std::printf("Can't open file \"%s\"\n", o.in.c_str());
        std::string line;
        Experiment e;
        while (std::getline(in, line))
            if (ParseLine(line, e)) suite.push_back(e);
    }
    El::Grid g;
    std::printf("Grid: %dx%d\n\n", g.Height(), g.Width());
    bool ok = true;
    std::vector<std::vector<double>> results;
    try {
        for (const auto& e : suite)
            results.push_back(e.dev == El::Device::GPU ? Dispatch<El::Device::GPU>(e, o, g, ok)
                                                       : Dispatch<El::Device::CPU>(e, o, g, ok));
    } catch (const std::exception& ex) {
        std::fprintf(stderr, "error: %s\n", ex.what());
        return 1;
    }
    if (!o.out.empty()) {
        std::ofstream out(o.out);
        if (!out) throw std::runtime_error("Bad news: " + o.out);
        for (size_t i = 0; i < suite.size(); ++i) {
            const auto& e = suite[i];
            out << (e.dev == El::Device::GPU ? "GPU" : "CPU") << ':' << TypeName(e.type) << ':'
                << OrientName(e.oa) << ':' << OrientName(e.ob) << ':' << e.alg_name << ':' << e.m << ':' << e.n
                << ':' << e.k << ':' << e.nb;
            for (double t : results[i]) out << ':' << t;
            out << '\n';
        }
    }
    El::Finalize();
    return ok ? 0 : 1;
}
