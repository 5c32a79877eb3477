// qi_ec_driver -- file-level integration driver over the product's C++ API
// (include/qi_fec.hpp), with the command line and on-disk format of
// QuadIron's test/ec_driver.cpp (RS-FNT flavours only):
//
//   qi_ec_driver -e rs-fnt|rs-fnt-sys -w 2 -n K -m M -p PREFIX -c|-r [-t] [-v]
//
//   -c  create PREFIX.cNN (+ PREFIX.cNN.props, text Properties) from the data
//       files PREFIX.dNN through encode_streams_vertical
//       (test/ec_driver.cpp:104-173)
//   -r  repair the missing data files from the coding files present (and
//       their .props) through decode_streams_vertical, then re-create every
//       coding file (test/ec_driver.cpp:179-286, 430-457)
//   -t  print SYSTEMATIC / NON_SYSTEMATIC and exit 1 (as the reference)
//
// File names: PREFIX.d<i> / PREFIX.c<i>, zero padded to the digits of
// n_data - 1 / n_outputs - 1 (test/ec_driver.cpp:87-98, 589); pkt_size 1024
// (test/ec_driver.cpp:430-437).  tests/test_ec_files.py drives it through
// the scenarios of scripts/test_ec.sh.  Test infrastructure, not product.
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iomanip>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/qi_fec.hpp"

namespace {

int vflag = 0;
int data_zpad = 1, coding_zpad = 1;
std::string prefix;

[[noreturn]] void usage()
{
    std::cerr << "usage: qi_ec_driver -e rs-fnt|rs-fnt-sys -w 2 -n n_data -m "
                 "n_parities -p prefix -c|-r [-t] [-v]\n";
    std::exit(EXIT_FAILURE);
}

unsigned count_digits(unsigned number)
{
    unsigned digits = 0;
    while (number) {
        number /= 10;
        digits++;
    }
    return digits;
}

std::string filename(char type, int zpad, unsigned part, const std::string& ext = "")
{
    std::ostringstream oss;
    oss << prefix << "." << type << std::setfill('0') << std::setw(zpad) << part << ext;
    return oss.str();
}

bool exists(const std::string& f)
{
    return access(f.c_str(), F_OK) == 0;
}

void create_coding_files(qi::fec::RsFnt& fec)
{
    std::vector<std::istream*> d(fec.n_data, nullptr);
    std::vector<std::ostream*> c(fec.n_outputs, nullptr);
    std::vector<qi::Properties> props(fec.n_outputs);
    for (unsigned i = 0; i < fec.n_data; i++) {
        auto* f = new std::ifstream(filename('d', data_zpad, i), std::ios::binary);
        if (f->fail()) {
            std::cerr << "cannot open data file " << filename('d', data_zpad, i) << "\n";
            std::exit(EXIT_FAILURE);
        }
        d[i] = f;
    }
    for (unsigned i = 0; i < fec.n_outputs; i++) {
        auto* f = new std::ofstream(filename('c', coding_zpad, i), std::ios::binary);
        if (f->fail()) {
            std::cerr << "cannot create coding file\n";
            std::exit(EXIT_FAILURE);
        }
        c[i] = f;
    }
    fec.encode_streams_vertical(d, c, props);
    for (auto* f : d)
        delete f;
    for (unsigned i = 0; i < fec.n_outputs; i++) {
        std::ofstream pf(filename('c', coding_zpad, i, ".props"));
        pf << props[i];
        delete c[i];
    }
}

bool repair_data_files(qi::fec::RsFnt& fec)
{
    std::vector<std::istream*> d(fec.n_data, nullptr), c(fec.n_outputs, nullptr);
    std::vector<std::ostream*> r(fec.n_data, nullptr);
    std::vector<qi::Properties> props(fec.n_outputs);
    for (unsigned i = 0; i < fec.n_data; i++) {
        const std::string f = filename('d', data_zpad, i);
        if (!exists(f)) {
            if (vflag)
                std::cerr << f << " is missing\n";
            r[i] = new std::ofstream(f, std::ios::binary);
        } else {
            d[i] = new std::ifstream(f, std::ios::binary);
        }
    }
    for (unsigned i = 0; i < fec.n_outputs; i++) {
        const std::string f = filename('c', coding_zpad, i);
        if (exists(f))
            c[i] = new std::ifstream(f, std::ios::binary);
        else if (vflag)
            std::cerr << f << " is missing\n";
        const std::string pf = filename('c', coding_zpad, i, ".props");
        if (exists(pf)) {
            std::ifstream in(pf);
            in >> props[i];
        }
    }
    const bool ok = fec.decode_streams_vertical(d, c, props, r);
    for (auto* f : d)
        delete f;
    for (auto* f : c)
        delete f;
    for (auto* f : r)
        delete f;
    return ok;
}

}  // namespace

int main(int argc, char** argv)
{
    int opt, cflag = 0, rflag = 0, tflag = 0;
    int n_data = -1, n_parities = -1, word_size = 0;
    std::string type;
    while ((opt = getopt(argc, argv, "n:m:p:crve:w:t")) != -1) {
        switch (opt) {
        case 'e':
            type = optarg;
            break;
        case 'w':
            word_size = std::atoi(optarg);
            break;
        case 'v':
            vflag = 1;
            break;
        case 'c':
            cflag = 1;
            break;
        case 'r':
            rflag = 1;
            break;
        case 'n':
            n_data = std::atoi(optarg);
            break;
        case 'm':
            n_parities = std::atoi(optarg);
            break;
        case 'p':
            prefix = optarg;
            break;
        case 't':
            tflag = 1;
            break;
        default:
            usage();
        }
    }
    if ((type != "rs-fnt" && type != "rs-fnt-sys") || n_data < 1 || n_parities < 1 ||
        prefix.empty() || !(cflag || rflag || tflag))
        usage();
    data_zpad = static_cast<int>(count_digits(static_cast<unsigned>(n_data - 1)));
    try {
        qi::fec::RsFnt fec(type == "rs-fnt-sys" ? qi::fec::FecType::SYSTEMATIC
                                                : qi::fec::FecType::NON_SYSTEMATIC,
                           static_cast<unsigned>(word_size), static_cast<unsigned>(n_data),
                           static_cast<unsigned>(n_parities), 1024);
        coding_zpad = static_cast<int>(count_digits(fec.n_outputs - 1));
        if (tflag) {
            std::cout << (fec.type == qi::fec::FecType::SYSTEMATIC ? "SYSTEMATIC\n"
                                                                   : "NON_SYSTEMATIC\n");
            return EXIT_FAILURE;
        }
        if (rflag && !repair_data_files(fec)) {
            std::cerr << "repair: fewer than n_data fragments\n";
            return EXIT_FAILURE;
        }
        create_coding_files(fec);
        std::cerr << "enc," << fec.n_encode_ops << "," << fec.total_enc_usec << "us,dec,"
                  << fec.n_decode_ops << "," << fec.total_dec_usec << "us\n";
    } catch (const std::exception& e) {
        std::cerr << "qi_ec_driver: " << e.what() << "\n";
        return EXIT_FAILURE;
    }
    return EXIT_SUCCESS;
}
