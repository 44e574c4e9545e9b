"""One decoder-GEMM variant only (for rocprofv3 --pmc passes): python gemm_one.py <variant>"""
import sys
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.abspath(__file__)))
import gemm_bench  # noqa: E402
gemm_bench.main(sys.argv[1])
