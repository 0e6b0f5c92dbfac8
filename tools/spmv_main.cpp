// spmv_main.cpp -- reference-shaped driver for the MI355X engine.
//
// Same flow and report as the reference driver (src/main.cpp:17-209):
//   srand(3); load .mtx; x, y = CreateRandomVector; OptimizeProblem once;
//   VERIFY: SpMV + VerifyResult twice; warm-up doubling the loop count until
//   >= 1 s; 10 trials of `loop` calls keeping the minimum mean; print the
//   "++++ ... ----" key/value block (parsable by the reference log/format.cpp)
// with GPU additions: AchievedGB/s against the plan's algorithmic bytes and
// the MI355X 8 TB/s HBM roofline.
//
// Usage: spmv <matrix.mtx> [--format crs|ell|ss|dia|hyb|css|coo|jds|bin|auto] [--resident]
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>

#include "opt_hip.h"

int main(int argc, char **argv) {
    srand(3);  // src/main.cpp:18
    if (argc < 2) {
        std::printf("Usage: %s <matrix> [--format crs|ell|ss|dia|hyb|css|coo|jds|bin|auto] [--resident]\n", argv[0]);
        return 1;
    }
    const std::string matFile = argv[1];
    for (int i = 2; i < argc; ++i) {
        if (!std::strcmp(argv[i], "--format") && i + 1 < argc) setenv("SPMV_HIP_FORMAT", argv[++i], 1);
        else if (!std::strcmp(argv[i], "--resident")) setenv("SPMV_HIP_X_RESIDENT", "1", 1);
    }
    SpMat A;
    std::cerr << "Loading sparse matrix " << matFile << " ... ";
    LoadSparseMatrix(A, matFile);
    std::cerr << "done." << std::endl;
    Vec x = CreateRandomVector(A.nCol);
    Vec y = CreateRandomVector(A.nRow);
    SpMatOpt A_opt;
    VecOpt x_opt;
    std::cerr << "Optimizing ... ";
    OptimizeProblem(A, x, A_opt, x_opt);
    std::cerr << "done." << std::endl;

    for (int i = 0; i < 2; ++i) {  // src/main.cpp:40-56
        SpMV(A_opt, x_opt, y);
        std::cerr << "Verifying " << i << " ... ";
        if (!VerifyResult(A, x, y)) {
            std::printf("*** invalid result ***\n");
            return 1;
        }
        std::cerr << "done." << std::endl;
    }

    int loop = 1;  // src/main.cpp:58-71
    std::cerr << "Calculating SpMV ... ";
    const double t0 = GetTimeBySec();
    do {
        for (int i = 0; i < loop; ++i) SpMV(A_opt, x_opt, y);
        loop *= 2;
    } while (GetTimeBySec() - t0 < 1.0);
    double best = 0;  // src/main.cpp:79-102
    for (int t = 0; t < 10; ++t) {
        const double s = GetTimeBySec();
        for (int i = 0; i < loop; ++i) SpMV(A_opt, x_opt, y);
        const double e = (GetTimeBySec() - s) / loop;
        if (t == 0 || e < best) best = e;
    }
    std::cerr << "done." << std::endl;

    spmv_plan_info_t info;
    spmv_plan_info(A_opt.plan, &info);
    static const char *names[] = {"AUTO", "CRS", "ELL", "SS", "DIA", "HYB", "CSS", "COO", "JDS", "BIN"};
    const double gflops = (double)A.nNnz * 2.0 / best / 1e9;
    const double gbs = (double)info.algo_bytes / best / 1e9;
    std::printf("++++++++++++++++++++++++++++++++++++++++\n");
    std::printf("%25s\t%s\n", "Architecture", "GPU");
    std::printf("%25s\t%s\n", "MatrixFormat", names[info.format]);
    std::printf("%25s\t%s\n", "Kernel", info.kernel);
    std::printf("%25s\t%s\n", "Matrix", GetBasename(matFile).c_str());
    std::printf("%25s\t%s\n", "MatrixPath", matFile.c_str());
    std::printf("%25s\t%lf\n", "Performance(GFLOPS)", gflops);
    std::printf("%25s\t%lf\n", "AchievedGB/s", gbs);
    std::printf("%25s\t%lf\n", "RooflineFrac", gbs / 8000.0);
    std::printf("%25s\t%d\n", "nRow", A.nRow);
    std::printf("%25s\t%d\n", "nCol", A.nCol);
    std::printf("%25s\t%d\n", "nNnz", A.nNnz);
    std::printf("%25s\t%d\n", "nGPU", 1);
    std::printf("%25s\t%s\n", "XResident", getenv("SPMV_HIP_X_RESIDENT") ? "1" : "0");
    std::printf("----------------------------------------\n");
    SpMVRelease(A_opt);
    return 0;
}
