// convection_diffusion — steady convection-diffusion-reaction MMS solve through the MFEM-shaped
// host API (cdfem_mfem.hpp) on the MI355X kernels.
//
// Follows the hot-path sequence of myapps/convection_diffusion/linear_convection_diffusion_2D.cpp
// (:300-392): mesh + H1 space, all-boundary Dirichlet, Diffusion + Convection + Mass integrators,
// DomainLF forcing, boundary projection of the exact solution, FormLinearSystem, a
// PetscLinearSolver configured from a PETSc options file (Input/petsc.opts keys), solve,
// RecoverFEMSolution, L2 error.  The problem is the reference's MMS u = sin(n pi x) sin(m pi y)
// (:159-170), extended with sin(l pi z) in 3D; the forcing is the reference's (:174-205) plus the
// z terms.  Configuration comes from the command line instead of YAML (out of scope).
//
//   convection_diffusion [-d dim] [-n elems | -mesh file.msh] [-p order] [-k kappa] [-s reaction]
//                        [-c cx,cy,cz] [-m n,m,l] [-opts petsc.opts] [-pl print_level]
// Output (stdout, one "key value" per line): dofs, iterations, converged, final_norm, l2_abs,
// l2_rel, solve_seconds.  Exit code 3 on error (as the reference drivers, :435-442).
#include <cmath>
#include <cstdio>
#include <cstring>
#include <exception>
#include <string>

#include "cdfem_mfem.hpp"

using namespace cdfem::mfem;

namespace {

struct Params {
    int dim = 2, n = 16, order = 2, print_level = 0;
    double kappa = 0.1, reaction = 1.0, c[3] = {1.0, -2.0, 0.5};
    int modes[3] = {3, 3, 3};
    std::string opts, mesh;
};

class ExactSolution : public Coefficient {
public:
    ExactSolution(int dim, const int *m) : dim_(dim), m_{m[0], m[1], m[2]} {}
    real_t Eval(ElementTransformation &T, const IntegrationPoint &ip) override
    {
        Vector x;
        T.Transform(ip, x);
        double u = std::sin(m_[0] * M_PI * x[0]) * std::sin(m_[1] * M_PI * x[1]);
        if (dim_ == 3) u *= std::sin(m_[2] * M_PI * x[2]);
        return u;
    }

private:
    int dim_;
    int m_[3];
};

// f = -kappa Lap u + c . grad u + s u for the product of sines
class Forcing : public Coefficient {
public:
    explicit Forcing(const Params &p) : p_(p) {}
    real_t Eval(ElementTransformation &T, const IntegrationPoint &ip) override
    {
        Vector x;
        T.Transform(ip, x);
        const int d = p_.dim;
        double s[3] = {1, 1, 1}, c[3] = {0, 0, 0}, k2 = 0.0;
        for (int i = 0; i < d; ++i) {
            const double a = p_.modes[i] * M_PI;
            s[i] = std::sin(a * x[i]);
            c[i] = a * std::cos(a * x[i]);
            k2 += a * a;
        }
        const double u = s[0] * s[1] * s[2];
        double conv = 0.0;
        for (int i = 0; i < d; ++i) {
            double g = c[i];
            for (int j = 0; j < d; ++j)
                if (j != i) g *= s[j];
            conv += p_.c[i] * g;
        }
        return p_.kappa * k2 * u + conv + p_.reaction * u;
    }

private:
    const Params &p_;
};

void parse_triplet(const char *s, double *out)
{
    std::sscanf(s, "%lf,%lf,%lf", &out[0], &out[1], &out[2]);
}

Params parse(int argc, char **argv)
{
    Params p;
    for (int i = 1; i + 1 < argc; i += 2) {
        const std::string k = argv[i];
        const char *v = argv[i + 1];
        if (k == "-d") p.dim = std::atoi(v);
        else if (k == "-n") p.n = std::atoi(v);
        else if (k == "-p") p.order = std::atoi(v);
        else if (k == "-k") p.kappa = std::atof(v);
        else if (k == "-s") p.reaction = std::atof(v);
        else if (k == "-c") parse_triplet(v, p.c);
        else if (k == "-m") std::sscanf(v, "%d,%d,%d", &p.modes[0], &p.modes[1], &p.modes[2]);
        else if (k == "-opts") p.opts = v;
        else if (k == "-mesh") p.mesh = v;
        else if (k == "-pl") p.print_level = std::atoi(v);
        else throw std::invalid_argument("unknown option " + k);
    }
    if (p.dim != 2 && p.dim != 3) throw std::invalid_argument("-d must be 2 or 3");
    return p;
}

}  // namespace

int main(int argc, char **argv)
{
    try {
        const Params prm = parse(argc, argv);
        MFEMInitializePetsc(&argc, &argv, prm.opts.empty() ? nullptr : prm.opts.c_str(), nullptr);

        // -mesh: a gmsh file as in the reference's inputs (Input/input_2d.yaml: mesh_file), else a box
        Mesh mesh = !prm.mesh.empty() ? Mesh(prm.mesh.c_str(), 1, 1)
                    : prm.dim == 2   ? Mesh::MakeCartesian2D(prm.n, prm.n, Element::QUADRILATERAL)
                                     : Mesh::MakeCartesian3D(prm.n, prm.n, prm.n, Element::HEXAHEDRON);
        if (!prm.mesh.empty() && mesh.Dimension() != prm.dim)
            throw std::invalid_argument("-d does not match the mesh file's dimension");
        H1_FECollection fec(prm.order, prm.dim);
        ParFiniteElementSpace fespace(&mesh, &fec);

        Array<int> ess_bdr(mesh.bdr_attributes.Max());
        ess_bdr = 1;
        Array<int> ess_tdof_list;
        fespace.GetEssentialTrueDofs(ess_bdr, ess_tdof_list);

        ExactSolution exact(prm.dim, prm.modes);
        Forcing forcing(prm);
        Vector cvec(prm.dim);
        for (int i = 0; i < prm.dim; ++i) cvec[i] = prm.c[i];
        VectorConstantCoefficient convection(cvec);
        ConstantCoefficient kappa(prm.kappa), reaction(prm.reaction);

        ParBilinearForm a(&fespace);
        a.AddDomainIntegrator(new DiffusionIntegrator(kappa));
        a.AddDomainIntegrator(new ConvectionIntegrator(convection));
        a.AddDomainIntegrator(new MassIntegrator(reaction));
        a.Assemble();

        ParLinearForm b(&fespace);
        b.AddDomainIntegrator(new DomainLFIntegrator(forcing));
        b.Assemble();

        ParGridFunction u(&fespace);
        u = 0.0;
        u.ProjectBdrCoefficient(exact, ess_bdr);

        OperatorHandle Ah(Operator::Hypre_ParCSR);
        Vector X, B;
        a.FormLinearSystem(ess_tdof_list, u, b, Ah, X, B);

        HypreParMatrix *A_true = Ah.As<HypreParMatrix>();
        if (!A_true) throw std::runtime_error("Expected the constrained operator from FormLinearSystem");
        PetscParMatrix A_petsc(0, A_true, Operator::PETSC_MATAIJ);
        PetscLinearSolver solver(A_petsc);
        solver.SetPrintLevel(prm.print_level);
        solver.Mult(B, X);

        a.RecoverFEMSolution(X, b, u);

        const int order_quad = std::max(2, 2 * prm.order + 3);
        const IntegrationRule *irs[Geometry::NumGeom] = {};
        for (int g = 0; g < Geometry::NumGeom; ++g) irs[g] = &IntRules.Get(g, order_quad);
        const double abs_l2 = u.ComputeL2Error(exact, irs);
        const double exact_l2 = ComputeGlobalLpNorm(2, exact, mesh, irs);

        std::printf("dofs %d\niterations %d\nconverged %d\nfinal_norm %.17g\nl2_abs %.17g\nl2_rel %.17g\n"
                    "solve_seconds %.6g\n",
                    fespace.GetTrueVSize(), solver.GetNumIterations(), solver.GetConverged() ? 1 : 0,
                    solver.GetFinalNorm(), abs_l2, exact_l2 > 1e-14 ? abs_l2 / exact_l2 : 0.0,
                    solver.GetSolveSeconds());
        if (!solver.GetConverged()) {
            std::fprintf(stderr, "solver did not converge: iterations=%d residual=%g\n",
                         solver.GetNumIterations(), solver.GetFinalNorm());
            return 3;
        }
        MFEMFinalizePetsc();
        return 0;
    } catch (const std::exception &e) {
        std::fprintf(stderr, "error: %s\n", e.what());
        return 3;
    }
}
