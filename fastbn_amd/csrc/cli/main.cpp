// main.cpp -- drop-in for `./BayesianNetwork -a 0|2 ...` (src/main.cpp:17-201, src/Parameter.cpp:6-107):
// same flags, defaults and "../dataset/" path prefix; -a 0 (PC-stable) and -a 2 (junction tree)
// run on the GPU.  Extra flags: --device N, --gpus G (devices N .. N + G - 1, RCCL: MultiGpu.h),
// --depth D (PC-stable max depth, reference default 1000).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>

#include "JunctionTree.h"
#include "PCStable.h"
#include "fastbn.h"

int main(int argc, char **argv) {
    int algorithm = 2, num_threads = 1, group_size = 1, device = 0, depth = 1000, gpus = 1;
    std::string net_file = "alarm/alarm.xml", ref_net_file = "alarm/alarm.bif",
                train_set_file = "alarm/alarm_s5000.txt", test_set_file = "alarm/testing_alarm_1k_p20",
                pt_file = "alarm/alarm_1k_pt", prefix = "../dataset/";
    int i;
    for (i = 1; i < argc && argv[i][0] == '-'; i++) {
        std::string a = argv[i];
        if (a == "--device" && i + 1 < argc) { device = atoi(argv[++i]); continue; }
        if (a == "--gpus" && i + 1 < argc) { gpus = atoi(argv[++i]); continue; }
        if (a == "--depth" && i + 1 < argc) { depth = atoi(argv[++i]); continue; }
        if (a == "--prefix" && i + 1 < argc) { prefix = argv[++i]; continue; }
        switch (argv[i][1]) {
        case 'h':
            std::cout << "Usage: ./BayesianNetwork [-a 0|2] [-t threads] [-g group] [-f0 net] [-f1 refnet] "
                         "[-f2 train] [-f3 test] [-f4 pt] [--device N] [--gpus G] [--depth D] [--prefix DIR]" << std::endl;
            return 0;
        case 'a': algorithm = atoi(argv[++i]); break;
        case 't': num_threads = atoi(argv[++i]); break;
        case 'g': group_size = atoi(argv[++i]); break;
        case 'q': case 'm': case 'l': case 'd': ++i; break;  // sampling-algorithm flags: accepted
        case 'f':
            switch (argv[i][2]) {
            case '0': net_file = argv[++i]; break;
            case '1': ref_net_file = argv[++i]; break;
            case '2': train_set_file = argv[++i]; break;
            case '3': test_set_file = argv[++i]; break;
            case '4': pt_file = argv[++i]; break;
            }
            break;
        default:
            printf("\n Unrecognized option %s!\n", argv[i]);
            return 0;
        }
    }
    net_file = prefix + net_file;
    ref_net_file = prefix + ref_net_file;
    train_set_file = prefix + train_set_file;
    test_set_file = prefix + test_set_file;
    pt_file = prefix + pt_file;

    if (algorithm == 0) {
        std::cout << "===============================" << std::endl
                  << "Algorithm: PC-stable for structure learning, #threads = " << num_threads << std::endl
                  << "group size = " << group_size << std::endl
                  << "\treference BN: " << ref_net_file << std::endl
                  << "\tsample set: " << train_set_file << std::endl
                  << "===============================" << std::endl;
        fbn_dataset *ds = nullptr;
        if (fbn_dataset_load_csv(train_set_file.c_str(), &ds)) {
            fprintf(stderr, "Error: %s\n", fbn_last_error());
            return 1;
        }
        PCStable pc(0.05, depth, device, gpus);
        pc.StructLearnCompData(ds, group_size, num_threads, false, false);
        fbn_dataset_destroy(ds);
        std::cout << "SHD = " << pc.GetSHD(ref_net_file) << std::endl;
    } else if (algorithm == 2) {
        std::cout << "===============================" << std::endl
                  << "Algorithm: junction tree (JT) for exact inference, #threads = " << num_threads << std::endl
                  << "\tBN: " << net_file << std::endl
                  << "\ttesting set: " << test_set_file << std::endl
                  << "\treference potential table: " << pt_file << std::endl
                  << "===============================" << std::endl;
        fbn_network *net = nullptr;
        if (fbn_network_load_xmlbif(net_file.c_str(), &net)) {
            fprintf(stderr, "Error: %s\n", fbn_last_error());
            return 1;
        }
        int n = 0;
        fbn_network_num_nodes(net, &n);
        TestSet tester;
        if (tester.Load(test_set_file, n)) {
            fprintf(stderr, "Error: %s\n", fbn_last_error());
            return 1;
        }
        double accuracy;
        {
            JunctionTree jt(net, &tester, device, gpus);
            accuracy = jt.EvaluateAccuracy(pt_file, num_threads);
        }
        std::cout << "accuracy = " << accuracy << std::endl;
        fbn_network_destroy(net);
    } else if (algorithm >= 0 && algorithm <= 11) {
        std::cout << "This algorithm is not on the accelerated path of this build (only -a 0 and -a 2)." << std::endl;
    } else {
        std::cout << "\tError! Please give the right value of -a to specify the functionality/algorithm" << std::endl;
    }
    return 0;
}
