"""CPU: the reference harness flags (utils/parameters.py) parse as the reference's, plus the README's
spellings the reference parser rejects (README.md:107,117; SURVEY.md section 5 probe P5)."""
import pytest

from xsdeepfwfm_deprecated_amd.cli import get_parser


def test_defaults_match_reference_parser():
    p = get_parser().parse_args([])
    # utils/parameters.py defaults
    assert (p.use_fwfm, p.use_deep, p.use_lw, p.use_fwlw, p.use_fm) == (1, 1, 1, 0, 0)
    assert (p.embedding_size, p.deep_nodes, p.h_depth) == (10, 400, 3)
    assert (p.batch_size, p.learning_rate, p.l2) == (2048, 1e-3, 3e-7)
    assert (p.emb_bag, p.qr_emb, p.qr_collisions, p.qr_threshold) == (0, 0, 4, 200)
    assert p.time_on_cuda == 0


@pytest.mark.parametrize("argv", [["-emb_bag", "1", "-qr_emb", "1"],
                                  ["-embedding_bag", "1", "-qr_flag", "1"],
                                  ["-embedding_bag", "1", "-qr_emb", "1"]])
def test_readme_and_parser_spellings_are_the_same_flags(argv):
    p = get_parser().parse_args(argv)
    assert p.emb_bag == 1 and p.qr_emb == 1
    assert not hasattr(p, "embedding_bag") and not hasattr(p, "qr_flag")


def test_readme_pruning_command_parses():
    # README.md:89 (BASELINE configs[3]) as written there
    p = get_parser().parse_args("-l2 6e-7 -n_epochs 10 -warm 2 -prune 1 -sparse 0.90  -prune_deep 1 -prune_fm 1 "
                                "-prune_r 1 -use_fwlw 1 -emb_r 0.444 -emb_corr 1.".split())
    assert (p.prune, p.prune_r, p.sparse, p.emb_r) == (1, 1, 0.90, 0.444)
