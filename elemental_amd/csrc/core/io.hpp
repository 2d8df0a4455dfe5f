// El::Write / El::Read for DistMatrix in the reference's BINARY and BINARY_FLAT
// formats (src/io/Write.cpp:70-86, Write/Binary.hpp, Write/BinaryFlat.hpp,
// src/io/Read.cpp:71-120, Read/Binary.hpp, Read/BinaryFlat.hpp).
#pragma once
#include <string>
#include "distmatrix.hpp"

namespace elx {

// FileFormat ordinals of include/El/core/types.hpp:543-559
enum FileFormat : int { FILE_AUTO = 0, FILE_BINARY = 3, FILE_BINARY_FLAT = 4 };

// BINARY: [Int height][Int width][column-major data]; BINARY_FLAT: the data only.
// intBytes = sizeof(El::Int): 4 (the reference's default build) or 8
// (Hydrogen_USE_64BIT_INTS).  16-bit matrices travel as float, as the
// reference's gpu_half_type overloads do (Write.cpp:88-107, Read.cpp:124-135).
void Write(const DistMatrix& A, const std::string& basename, int format, int intBytes);
void Read(DistMatrix& A, const std::string& filename, int format, int intBytes);

}  // namespace elx
