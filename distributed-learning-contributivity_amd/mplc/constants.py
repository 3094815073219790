"""Constants of the coalition path (values are semantics: mplc/constants.py:7-43)."""

# ML constants
DEFAULT_BATCH_SIZE = 256                       # evaluate() batch size (mplc/constants.py:7)
MAX_BATCH_SIZE = 2 ** 20
DEFAULT_GRADIENT_UPDATES_PER_PASS_COUNT = 8
PATIENCE = 10                                  # early stopping patience (mplc/constants.py:10)
DEFAULT_BATCH_COUNT = 20
DEFAULT_EPOCH_COUNT = 40

# Contributivity methods names (mplc/constants.py:28-43)
CONTRIBUTIVITY_METHODS = [
    "Shapley values",
    "Independent scores",
    "TMCS",
    "ITMCS",
    "IS_lin_S",
    "IS_reg_S",
    "AIS_Kriging_S",
    "SMCS",
    "WR_SMC",
    "Federated SBS linear",
    "Federated SBS quadratic",
    "Federated SBS constant",
    "LFlip",
    "PVRL",
]

# Datasets' tags
MNIST = "mnist"
CIFAR10 = "cifar10"
TITANIC = "titanic"
SUPPORTED_DATASETS_NAMES = [MNIST, CIFAR10, TITANIC]

EXPERIMENTS_FOLDER_NAME = "experiments"
INFO_LOGGING_FILE_NAME = "info.log"
DEBUG_LOGGING_FILE_NAME = "debug.log"
