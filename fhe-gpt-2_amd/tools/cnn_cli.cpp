// ./cnn LAYER DATASET START END -- the reference's driver (cnn_ckks/run/run_cnn.cpp:8-27) over the
// MI355X library: argument checks and banner as the reference, then ResNet_cifar10_seal_sparse,
// which writes ../../result/resnet{L}_cifar10_image{id}.txt and _label_{start}_{end}.
#include "mhe_resnet.h"

#include <cstdlib>
#include <iostream>
#include <stdexcept>

int main(int argc, char **argv)
{
    if (argc < 5)
    {
        std::cerr << "usage: cnn LAYER DATASET START END" << std::endl;
        return 2;
    }
    const int layer = std::atoi(argv[1]);
    const int dataset = std::atoi(argv[2]);
    const int start = std::atoi(argv[3]);
    const int end = std::atoi(argv[4]);
    if (start < 0 || start >= 10000) throw std::invalid_argument("start number is not correct");
    if (end < 0 || end >= 10000) throw std::invalid_argument("end number is not correct");
    if (start > end) throw std::invalid_argument("start number is larger than end number");
    std::cout << "model: ResNet-" << layer << std::endl;
    std::cout << "dataset: CIFAR-" << dataset << std::endl;
    std::cout << "start image: " << start << std::endl;
    std::cout << "end image: " << end << std::endl;
    if (dataset == 10) ResNet_cifar10_seal_sparse((std::size_t)layer, (std::size_t)start, (std::size_t)end);
    return 0;
}
