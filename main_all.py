"""Entry point of the reference (main_all.py), on the MI355X engine: parse the same flags, read the
dataset (native ingest), build DeepFMs, fit (HIP training step; with -use_cuda 0 the host kernels), reload the
saved weights, report the model size and run the benchmark on the test split (on the device with
-time_on_cuda 1, else the host kernels' thread sweep).

    python main_all.py -dataset tiny-criteo -n_epochs 2 [-data_root DIR]
"""
import os
import random
from datetime import datetime

import numpy as np
import torch

from xsdeepfwfm_deprecated_amd.cli import get_logger, get_model, get_parser, load_model_dic
from xsdeepfwfm_deprecated_amd.data import get_dataset


def main(argv=None):
    pars = get_parser().parse_args(argv)
    np.random.seed(pars.random_seed)
    random.seed(pars.random_seed)
    torch.manual_seed(pars.random_seed)
    torch.cuda.manual_seed(pars.random_seed)

    os.makedirs("./saved_models", exist_ok=True)
    save_model_name = "./saved_models/" + pars.c + "_l2_" + str(pars.l2) + "_dt_" + pars.dataset
    if pars.prune:
        save_model_name += "_sparse_" + str(pars.sparse) + "_seed_" + str(pars.random_seed)
    if pars.emb_bag and not pars.qr_emb:
        save_model_name += "_emb_bag"
    if pars.qr_emb:
        save_model_name += "_qr"
    save_model_name += "_" + datetime.now().strftime("%Y%m%d%H%M%S")

    logger = get_logger(save_model_name[14:])
    logger.info(pars)
    logger.info("GET DATASET")
    field_size, train_dict, valid_dict, test_dict = get_dataset(pars, root=pars.data_root)

    cuda = bool(pars.use_cuda) and torch.cuda.is_available()
    model = get_model(field_size=field_size, cuda=cuda, feature_sizes=train_dict["feature_sizes"], pars=pars,
                      logger=logger)
    if cuda:
        model = model.cuda()
    model.fit(train_dict["index"], train_dict["value"], train_dict["label"], valid_dict["index"],
              valid_dict["value"], valid_dict["label"], prune=pars.prune, prune_fm=pars.prune_fm,
              prune_r=pars.prune_r, prune_deep=pars.prune_deep, save_path=save_model_name, emb_r=pars.emb_r,
              emb_corr=pars.emb_corr, early_stopping=False)

    # measurements: the reference rebuilds the model (on the device with -time_on_cuda 1, else on the CPU),
    # reloads the saved weights, reports the size and benchmarks the test split (main_all.py:56-63); on the CPU
    # the host kernels run the reference's 1- / 4-thread sweep (model/DeepFMs.py:982-1009)
    on_dev = bool(pars.time_on_cuda) and torch.cuda.is_available()
    model = get_model(field_size=field_size, cuda=on_dev, feature_sizes=train_dict["feature_sizes"], pars=pars,
                      logger=logger)
    model = load_model_dic(model, save_model_name, sparse=pars.prune)
    if on_dev:
        model = model.cuda()
    model.print_size_of_model()
    logger.info("TEST DATASET")
    return model.run_benchmark(test_dict["index"], test_dict["value"], test_dict["label"], batch_size=8192,
                               cuda=on_dev)


if __name__ == "__main__":
    main()
