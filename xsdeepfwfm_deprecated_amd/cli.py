"""The reference harness around the model: utils/parameters.py (get_parser: the same flags and
defaults), utils/util.py (get_logger, get_model, load_model_dic).  `main_all.py` at the repo root is the
entry point that uses them."""
from __future__ import annotations

import argparse
import logging
import os
import sys

import torch

from .DeepFMs import DeepFMs


def get_parser():
    """utils/parameters.py:2-51 (flags, defaults and help as the reference) + -data_root."""
    p = argparse.ArgumentParser(description="Hyperparameter tuning and selection")
    a = p.add_argument
    a("-c", default="DeepFwFM", type=str, help="Models: FM, DeepFwFM ...")
    a("-use_cuda", default=1, type=int, help="Use CUDA or not")
    a("-gpu", default=0, type=int, help="GPU id")
    a("-n_epochs", default=8, type=int, help="Number of epochs")
    a("-numerical", default=13, type=int, help="Numerical features, 13 for Criteo")
    a("-use_multi", default="0", type=int, help="Use multiple CUDAs")
    a("-use_logit", default=0, type=int, help="Use Logistic regression")
    a("-use_fm", default=0, type=int, help="Use FM module or not")
    a("-use_fwlw", default=0, type=int, help="If to include FwFM linear weights or not")
    a("-use_lw", default=1, type=int, help="If to include FM linear weights or not")
    a("-use_ffm", default=0, type=int, help="Use FFM module or not")
    a("-use_fwfm", default=1, type=int, help="Use FwFM module or not")
    a("-use_deep", default=1, type=int, help="Use Deep module or not")
    a("-num_deeps", default=1, type=int, help="Number of deep networks")
    a("-deep_nodes", default=400, type=int, help="Nodes in each layer")
    a("-h_depth", default=3, type=int, help="Deep layers")
    a("-prune", default=0, type=int, help="Prune model or not")
    a("-prune_r", default=0, type=int, help="Prune r")
    a("-prune_deep", default=1, type=int, help="Prune Deep component")
    a("-prune_fm", default=1, type=int, help="Prune FM component")
    a("-emb_r", default=1., type=float, help="Sparse FM ratio over Sparse Deep ratio")
    a("-emb_corr", default=1., type=float, help="Sparse Corr ratio over Sparse Deep ratio")
    a("-sparse", default=0.9, type=float, help="Sparse rate")
    a("-warm", default=10, type=float, help="Warm up epochs before pruning")
    a("-ensemble", default=0, type=int, help="Ensemble models or not")
    a("-embedding_size", default=10, type=int, help="Embedding size")
    a("-batch_size", default=2048, type=int, help="Batch size")
    a("-random_seed", default=42, type=int, help="Random seed")
    a("-learning_rate", default=0.001, type=float, help="Learning rate")
    a("-momentum", default=0, type=float, help="Momentum")
    a("-l2", default=3e-7, type=float, help="L2 penalty")
    a("-dataset", default="criteo", type=str, help="Dataset to use",
      choices=["criteo", "tiny-criteo", "twitter", "ali", "avazu"])
    a("-save_model_path", default=0, type=str, help="Saved model path")
    a("-dynamic_quantization", default=0, type=int, help="Apply dynamic network quantization")
    a("-static_quantization", default=0, type=int, help="Apply static network quantization")
    a("-quantization_aware", default=0, type=int, help="Quantization Aware Training")
    a("-kd", default=0, type=int, help="Perform knowledge distillation")
    a("-loss_type", default="logloss", type=str, help="Used loss (should be logloss but for kd we need softmax)")
    # the README's spellings (-embedding_bag / -qr_flag, reference README.md:107,117) are rejected by the
    # reference parser (probe P5); both spellings are accepted here, same destination
    a("-emb_bag", "-embedding_bag", dest="emb_bag", default=0, type=int, help="Use embedding bag")
    a("-qr_emb", "-qr_flag", dest="qr_emb", default=0, type=int, help="Use QR Embeddings")
    a("-qr_operation", default="mult", type=str)
    a("-qr_collisions", default=4, type=int)
    a("-qr_threshold", default=200, type=int)
    a("-twitter_category", default="like", type=str, choices=["reply", "retweet", "retweet_comment", "like"])
    a("-time_on_cuda", default=0, type=int)
    a("-data_root", default=".", type=str, help="directory holding data/ (this engine's addition)")
    return p


def get_logger(filename=None, log_dir="./logs"):
    """utils/util.py:22-40 (stdout + ./logs/<name>.log)."""
    root = logging.getLogger("xsDeepFwFM")
    root.setLevel(logging.DEBUG)
    fmt = logging.Formatter("%(asctime)s - %(name)s - %(levelname)s - %(message)s")
    h = logging.StreamHandler(sys.stdout)
    h.setLevel(logging.DEBUG)
    h.setFormatter(fmt)
    root.addHandler(h)
    if filename:
        os.makedirs(log_dir, exist_ok=True)
        # string concatenation as the reference ('./logs/' + filename): main_all's name starts with '/'
        fh = logging.FileHandler(filename=log_dir + "/" + filename + ".log")
        fh.setLevel(logging.DEBUG)
        fh.setFormatter(fmt)
        root.addHandler(fh)
    root.propagate = False
    return root


def load_model_dic(model, model_file, sparse=False):
    """utils/util.py:43-53; files this engine wrote are plain state dicts (weights_only load)."""
    state_dict = torch.load(model_file, weights_only=True, map_location="cpu")
    if sparse:
        model.load_state_dict(state_dict, strict=False)  # the reference's to_sparse() result is discarded
    else:
        model.load_state_dict(state_dict)
    return model


def get_model(cuda, feature_sizes, pars, dynamic_quantization=False, static_quantization=False,
              quantization_aware=False, field_size=39, deep_nodes=400, h_depth=3, logger=None):
    """utils/util.py:56-73."""
    return DeepFMs(field_size=field_size, feature_sizes=feature_sizes, embedding_size=pars.embedding_size,
                   n_epochs=pars.n_epochs, verbose=False, use_cuda=cuda, use_fm=pars.use_fm, use_fwfm=pars.use_fwfm,
                   use_ffm=pars.use_ffm, use_deep=pars.use_deep, batch_size=pars.batch_size,
                   learning_rate=pars.learning_rate, weight_decay=pars.l2, momentum=pars.momentum,
                   sparse=pars.sparse, warm=pars.warm, h_depth=pars.h_depth, deep_nodes=pars.deep_nodes,
                   num_deeps=pars.num_deeps, numerical=pars.numerical, use_lw=pars.use_lw, use_fwlw=pars.use_fwlw,
                   use_logit=pars.use_logit, random_seed=pars.random_seed, quantization_aware=quantization_aware,
                   dynamic_quantization=dynamic_quantization, static_quantization=static_quantization,
                   loss_type=pars.loss_type, embedding_bag=pars.emb_bag, qr_flag=pars.qr_emb,
                   qr_operation=pars.qr_operation, qr_collisions=pars.qr_collisions, qr_threshold=pars.qr_threshold,
                   logger=logger)
